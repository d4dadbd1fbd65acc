set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=${V:-e62}
FCX_LIB=$PWD/my_compress_amd/lib/libfcx_$V.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_route.py -m "gpu and not slow" > gpurun_out/r06_ab3_tests.log 2>&1 || { tail -40 gpurun_out/r06_ab3_tests.log; exit 1; }
tail -2 gpurun_out/r06_ab3_tests.log
NO_TRANS=1 SETS="${SETS:-rand text runs mix|cur:0 e62:0 e72:0}" bash tools/gpu_r06_ab.sh
