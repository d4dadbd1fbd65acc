#!/bin/bash
# Development: register / scratch / LDS use of the kernels of one HIP source (gfx950), one line each.
#   tools/kres.sh <file.hip> [name-filter]
f=$1; flt=${2:-.}
cd "$(dirname "$f")" && hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -I. -c "$(basename "$f")" \
  -o /tmp/kres_$$.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk '/Function Name:/{n=$NF=="[-Rpass-analysis=kernel-resource-usage]"?$(NF-1):$NF}
       /VGPRs: /{v=$(NF-1)} /VGPRs Spill:/{s=$(NF-1)} /ScratchSize/{sc=$(NF-1)} /LDS Size/{l=$(NF-1); print n, "vgpr", v, "spill", s, "scratch", sc, "lds", l}' |
  c++filt | grep -E "$flt"
rm -f /tmp/kres_$$.o
