set -u
R=$PWD
export TMPDIR=/tmp
for leg in rand:4 mix:0; do
  IFS=: read kind seed <<< "$leg"
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pk6_$kind -o run --output-format csv -- python3 $R/tools/devbench.py --kind $kind --seed $seed --mib 1024 --reps 5 > $R/gpurun_out/pk6_$kind.log 2>&1) || exit 1
  f=$(find $R/gpurun_out/pk6_$kind -name "*kernel_stats.csv" | head -1)
  head -14 $f | cut -d, -f1-6
done
