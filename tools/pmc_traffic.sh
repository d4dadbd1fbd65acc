# HBM traffic per kernel launch from rocprofv3 PMC counters (separate passes per counter,
# --kernel-trace only): FETCH_SIZE and WRITE_SIZE for each leg name:kind:block of bench.py
set -u
R=$PWD; export TMPDIR=/tmp; cd /tmp
for leg in ${LEGS:-rand:rand:1048576 text:text:1048576 c3:text:262144 zeros:zeros:1048576 runs:runs:1048576}; do
  IFS=: read name kind block <<< "$leg"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d $R/gpurun_out/traffic_${name}_$ctr -o run --output-format csv -- python3 $R/bench.py --kind $kind --block $block --steps 2 --warmup 0 --no-cpu-baseline --no-text --no-verify --no-decode --no-host-path --no-lz78 --no-transition > $R/gpurun_out/traffic_${name}_$ctr.log 2>&1 || exit 1
  done
done
