# HBM traffic per kernel launch from rocprofv3 PMC counters (separate passes per counter,
# --kernel-trace only): FETCH_SIZE and WRITE_SIZE for the rand and text legs of bench.py
set -u
R=$PWD; export TMPDIR=/tmp; cd /tmp
for kind in rand text; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $R/gpurun_out/traffic_${kind}_$ctr -o run --output-format csv -- python3 $R/bench.py --kind $kind --steps 2 --warmup 0 --no-cpu-baseline --no-text --no-verify > $R/gpurun_out/traffic_${kind}_$ctr.log 2>&1 || exit 1
  done
done
