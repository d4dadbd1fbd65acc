# k_match phase-exit timing for $KINDS (default rand text dna)
set -u
for kind in ${KINDS:-rand text dna}; do
  case $kind in text) seed=3;; rand) seed=4;; runs) seed=5;; dna) seed=6;; *) seed=0;; esac
  timeout -k 10 120 python tools/matchphase.py --kind $kind --seed $seed --mib 1024 --reps 3 > gpurun_out/phase_$kind.log 2>&1 || exit 1
done
