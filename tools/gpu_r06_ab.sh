set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
for v in ${VARIANTS:-r05:0 cur:0 cur:7}; do
  lib=${v%%:*}; m=${v##*:}
  L=my_compress_amd/lib/libfcx.so; [ $lib != cur ] && L=my_compress_amd/lib/libfcx_$lib.so
  for k in ${KINDS:-rand}; do
    FCX_LIB=$PWD/$L timeout -k 10 200 python -u tools/devbench.py --kind $k --mode $m --mib 1024 --reps 20 > gpurun_out/ab_${lib}_${k}_$m.log 2>&1 || { tail -20 gpurun_out/ab_${lib}_${k}_$m.log; exit 1; }
    echo "== $lib $k mode $m: $(grep -E '^groups' gpurun_out/ab_${lib}_${k}_$m.log)"; grep -E "^   route|^   memset" gpurun_out/ab_${lib}_${k}_$m.log
  done
done
done
