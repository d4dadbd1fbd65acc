# A/B of library variants: devbench stage times per kind for lib/libfcx.so (A) and each
# lib/libfcx_<V>.so in $VARS (FCX_LIB), e.g. VARS="x y" KINDS="rand text" bash tools/gpu_ab.sh
set -u
for kind in ${KINDS:-rand text dna runs}; do
  case $kind in text) seed=3; chk="--check hl_text_1GiB";; rand) seed=4; chk="--check hl_rand_1GiB";;
    runs) seed=5; chk="--check cfg5b_runs_1GiB";; dna) seed=6; chk="";; zeros) seed=0; chk="--check cfg5a_zeros_1GiB";; esac
  timeout -k 10 200 python tools/devbench.py --kind $kind --seed $seed --mib 1024 $chk > gpurun_out/ab_A_$kind.log 2>&1 || exit 1
  for v in ${VARS:-b}; do
    FCX_LIB=$PWD/my_compress_amd/lib/libfcx_$v.so timeout -k 10 200 python tools/devbench.py --kind $kind --seed $seed --mib 1024 $chk > gpurun_out/ab_${v}_$kind.log 2>&1 || exit 1
  done
done
