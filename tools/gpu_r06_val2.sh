set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_route.py tests/test_gpu_parity.py -m "gpu and not slow" > gpurun_out/r06_val2_tests.log 2>&1 || { tail -50 gpurun_out/r06_val2_tests.log; exit 1; }
tail -2 gpurun_out/r06_val2_tests.log
NO_TRANS=1 SETS="${SETS:-rand text zeros runs mix|head:0 cur:0}" bash tools/gpu_r06_ab.sh
