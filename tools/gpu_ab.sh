# A/B of library variants: devbench stage times per kind for lib/libfcx.so (A) and each
# lib/libfcx_<V>.so in $VARS (FCX_LIB), e.g. VARS="x y" KINDS="rand text" bash tools/gpu_ab.sh
set -u
for kind in ${KINDS:-rand text dna runs}; do
  case $kind in text) seed=3;; rand) seed=4;; runs) seed=5;; dna) seed=6;; zeros) seed=0;; esac
  timeout -k 10 200 python tools/devbench.py --kind $kind --seed $seed --mib 1024 > gpurun_out/ab_A_$kind.log 2>&1 || exit 1
  for v in ${VARS:-b}; do
    FCX_LIB=$PWD/my_compress_amd/lib/libfcx_$v.so timeout -k 10 200 python tools/devbench.py --kind $kind --seed $seed --mib 1024 > gpurun_out/ab_${v}_$kind.log 2>&1 || exit 1
  done
done
