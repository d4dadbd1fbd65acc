# PMC passes over the compress pipeline (k_match focus); outputs under gpurun_out/pmc_<kind>_<set>
set -u
R=$PWD; export TMPDIR=/tmp; cd /tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY"
for kind in ${KINDS:-text rand}; do
  case $kind in text) seed=3;; rand) seed=4;; runs) seed=5;; dna) seed=6;; *) seed=0;; esac
  for set in A B; do
    eval "C=\$$set"
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d $R/gpurun_out/pmc_${kind}_$set -o run --output-format csv -- python3 $R/tools/devbench.py --kind $kind --seed $seed --mib 256 --reps 1 > $R/gpurun_out/pmc_${kind}_$set.log 2>&1 || exit 1
  done
done
