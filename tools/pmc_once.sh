set -u
R=$PWD
export TMPDIR=/tmp
for dbg in 0 2 1; do
  FCX_MATCH_DBG=$dbg timeout -k 10 120 python tools/devbench.py --kind text --seed 3 --mib 1024 --reps 2 > gpurun_out/abl_$dbg.log 2>&1 || exit 1
done
cd /tmp
rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY -d $R/gpurun_out/pmc1 -o run --output-format csv -- python3 $R/tools/devbench.py --kind text --seed 3 --mib 256 --reps 1 > $R/gpurun_out/pmc1.log 2>&1
echo pmc rc=$?
