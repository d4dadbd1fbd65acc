# k_match evidence: per-phase exit timing (tools/matchphase.py) and the SQ counter
# sets of tools/pmc_match.sh, for the kinds in $KINDS (default rand text runs)
set -u
R=$PWD
for kind in ${KINDS:-rand text runs}; do
  case $kind in text) seed=3;; rand) seed=4;; runs) seed=5;; *) seed=0;; esac
  timeout -k 10 120 python tools/matchphase.py --kind $kind --seed $seed --mib 1024 --reps 3 > gpurun_out/phase_$kind.log 2>&1 || exit 1
done
KINDS=${KINDS:-rand text runs} bash tools/pmc_match.sh || exit 1
python tools/pmc_summary.py gpurun_out > gpurun_out/pmc_match_summary.txt 2>&1 || true
