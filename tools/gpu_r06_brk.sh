set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_bench_ranks.py -m gpu > gpurun_out/r06_brk.log 2>&1; rc=$?; tail -5 gpurun_out/r06_brk.log; exit $rc
