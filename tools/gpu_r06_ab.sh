set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# A/B of library variants (FCX_LIB) on devbench legs: SETS = "kinds|variants;kinds|variants"
SETS=${SETS:-"rand zeros|r05:0 cur:0 cur:7;text|cur:0 sk8:0 sk16:0 sk32:0"}
IFS=';' read -ra sets <<< "$SETS"
for rep in 1 2; do
for set in "${sets[@]}"; do
  kinds=${set%%|*}; variants=${set##*|}
  for v in $variants; do
    lib=${v%%:*}; m=${v##*:}
    L=my_compress_amd/lib/libfcx.so; [ $lib != cur ] && L=my_compress_amd/lib/libfcx_$lib.so
    for k in $kinds; do
      FCX_LIB=$PWD/$L timeout -k 10 200 python -u tools/devbench.py --kind $k --mode $m --mib 1024 --reps 20 > gpurun_out/ab_${lib}_${k}_$m.log 2>&1 || { tail -20 gpurun_out/ab_${lib}_${k}_$m.log; exit 1; }
      echo "== $lib $k mode $m: $(grep -E '^groups' gpurun_out/ab_${lib}_${k}_$m.log)"; grep -E "^   route|^   memset" gpurun_out/ab_${lib}_${k}_$m.log | cut -c1-60
    done
  done
done
done
[ -n "${NO_TRANS:-}" ] && exit 0
timeout -k 10 300 python -u -c "
import json, torch, bench
print(json.dumps(bench.transition_leg(torch.device('cuda:0'))))
" > gpurun_out/r06_transition.log 2>&1 || { tail -20 gpurun_out/r06_transition.log; exit 1; }
tail -2 gpurun_out/r06_transition.log
