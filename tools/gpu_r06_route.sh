set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m "gpu and not slow" -k "key4 or units_routed or dense or dna or groups or random_inputs" > gpurun_out/r06_route_tests.log 2>&1 || { tail -40 gpurun_out/r06_route_tests.log; exit 1; }
tail -5 gpurun_out/r06_route_tests.log
for k in rand text runs dna zeros; do
  timeout -k 10 200 python -u tools/devbench.py --kind $k --mib 1024 --reps 10 > gpurun_out/r06_dev_$k.log 2>&1 || { tail -20 gpurun_out/r06_dev_$k.log; exit 1; }
  grep -E "groups|route|digest" gpurun_out/r06_dev_$k.log
done
