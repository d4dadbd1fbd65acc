# Development: SQ counter sets A and B over k_match<true> at two phase exits of tools/matchphase.py
# (e.g. with and without the candidate scan); outputs gpurun_out/pmcph_<tag>_<set>/
#   PHASES="+queries +q-nocand" KIND=text SEED=3 bash tools/pmc_phase.sh
set -u
R=$PWD; export TMPDIR=/tmp; cd /tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY"
i=0
for ph in ${PHASES:-+queries +q-nocand}; do
  i=$((i + 1))
  for set in A B; do
    eval "C=\$$set"
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d $R/gpurun_out/pmcph_${i}_$set -o run --output-format csv -- python3 $R/tools/matchphase.py --kind ${KIND:-text} --seed ${SEED:-3} --mib 256 --reps 1 --mode ${MODE:-0} --phases "$ph" > $R/gpurun_out/pmcph_${i}_$set.log 2>&1 || exit 1
  done
done
