# A/B/n timing: k_match and stage times of $KINDS under each library in $LIBS
# (in-tree builds under my_compress_amd/lib/, "-" = the default lib/libfcx.so)
set -u
for kind in ${KINDS:-text dna}; do
  case $kind in text) seed=3;; rand) seed=4;; runs) seed=5;; dna) seed=6;; *) seed=0;; esac
  for lib in ${LIBS:--}; do
    tag=$(basename $lib .so)
    if [ "$lib" = "-" ]; then
      timeout -k 10 200 python tools/devbench.py --kind $kind --seed $seed --mib 1024 > gpurun_out/abn_${tag}_$kind.log 2>&1 || exit 1
    else
      FCX_LIB=$PWD/$lib timeout -k 10 200 python tools/devbench.py --kind $kind --seed $seed --mib 1024 > gpurun_out/abn_${tag}_$kind.log 2>&1 || exit 1
    fi
  done
done
