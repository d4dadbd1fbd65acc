# checkpoint on one GPU: full -m gpu suite, default bench line, rocprofv3 kernel stats of the main leg
set -u
R=$PWD
timeout -k 10 800 python -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread > gpurun_out/tfull.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/tfull.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || exit 1
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_n1 -o run --output-format csv -- python3 $R/bench.py --no-text --no-decode --no-host-path > $R/gpurun_out/prof_n1.json 2> $R/gpurun_out/prof_n1.err) || exit 1
