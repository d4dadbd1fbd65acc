set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_route.py tests/test_gpu_parity.py -m "gpu and not slow" > gpurun_out/r06_val3_tests.log 2>&1 || { tail -50 gpurun_out/r06_val3_tests.log; exit 1; }
tail -2 gpurun_out/r06_val3_tests.log
for k in rand runs; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/v3_$k -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/devbench.py --kind $k --mib 1024 --reps 10 > $GRAFT_REPO_ROOT/gpurun_out/v3_$k.log 2>&1) || exit 1
  grep -h -E "classify|uniform" $GRAFT_REPO_ROOT/gpurun_out/v3_$k/run_kernel_stats.csv | cut -c1-160
  grep "^groups" gpurun_out/v3_$k.log
done
