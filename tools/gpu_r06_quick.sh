set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TESTS:-tests/test_gpu_route.py}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread $T -m "gpu and not slow" > gpurun_out/r06_quick_tests.log 2>&1 || { tail -40 gpurun_out/r06_quick_tests.log; exit 1; }
tail -3 gpurun_out/r06_quick_tests.log
for k in ${KINDS:-rand text}; do
  timeout -k 10 200 python -u tools/devbench.py --kind $k --mib 1024 --reps 10 > gpurun_out/r06_dev_$k.log 2>&1 || { tail -20 gpurun_out/r06_dev_$k.log; exit 1; }
  grep -E "groups|route|digest" gpurun_out/r06_dev_$k.log
done
