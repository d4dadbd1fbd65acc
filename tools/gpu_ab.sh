# A/B timing of lib/libfcx.so against an alternative in-tree build (FCX_LIB) on $KINDS
set -u
ALT=${ALT:-my_compress_amd/lib/libfcx_v.so}
for kind in ${KINDS:-text dna}; do
  case $kind in text) seed=3;; rand) seed=4;; runs) seed=5;; dna) seed=6;; *) seed=0;; esac
  timeout -k 10 200 python tools/devbench.py --kind $kind --seed $seed --mib 1024 > gpurun_out/ab_a_$kind.log 2>&1 || exit 1
  FCX_LIB=$PWD/$ALT timeout -k 10 200 python tools/devbench.py --kind $kind --seed $seed --mib 1024 > gpurun_out/ab_b_$kind.log 2>&1 || exit 1
done
