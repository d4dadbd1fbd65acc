set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r06_gpu_tests.log 2>&1 || { tail -60 gpurun_out/r06_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r06_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1 || { tail -20 gpurun_out/r06_smoke.log; exit 1; }
tail -1 gpurun_out/r06_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r06_bench_n1.json 2> gpurun_out/r06_bench_n1.err || { tail -30 gpurun_out/r06_bench_n1.err; exit 1; }
tail -c 1500 gpurun_out/r06_bench_n1.json
