set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TESTS:-tests/test_gpu_route.py}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread $T -m "gpu and not slow" > gpurun_out/r06_modes_tests.log 2>&1 || { tail -40 gpurun_out/r06_modes_tests.log; exit 1; }
tail -2 gpurun_out/r06_modes_tests.log
for km in ${RUNS:-rand:0 rand:7 text:0 text:5 zeros:0 zeros:6 mix:0}; do
  k=${km%%:*}; m=${km##*:}
  timeout -k 10 200 python -u tools/devbench.py --kind $k --mode $m --mib 1024 --reps 10 > gpurun_out/r06_dev_${k}_$m.log 2>&1 || { tail -20 gpurun_out/r06_dev_${k}_$m.log; exit 1; }
  echo "== $k mode $m"; grep -E "groups|   route|   memset" gpurun_out/r06_dev_${k}_$m.log
done
