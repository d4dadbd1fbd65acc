# PMC passes over the GPU decoder (development); outputs under gpurun_out/pmcd_<kind>_<set>
set -u
R=$PWD; export TMPDIR=/tmp; cd /tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY"
for kind in ${KINDS:-zeros rand}; do
  case $kind in text) seed=3;; rand) seed=4;; runs) seed=5;; *) seed=0;; esac
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $A -d $R/gpurun_out/pmcd_${kind}_A -o run --output-format csv -- python3 $R/tools/decbench.py --kind $kind --seed $seed --mib ${PMC_MIB:-128} --reps 1 > $R/gpurun_out/pmcd_${kind}_A.log 2>&1 || exit 1
done
