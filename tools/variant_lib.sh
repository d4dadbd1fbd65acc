# Development: build my_compress_amd/lib/libfcx_<name>.so with one source (default fcx_match) replaced by
# a variant (the other objects from the current build), for tools/gpu_ab.sh; EXTRA: more compiler flags.
#   [EXTRA="-mllvm ..."] bash tools/variant_lib.sh name file.hip [fcx_parse]
set -eu
name=$1; src=$(readlink -f $2); tgt=${3:-fcx_match}
cd "$(dirname "$0")/../my_compress_amd/csrc"
make -s
mkdir -p build/v_$name
cp $src ./fm_v_$name.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I../../include -I. ${EXTRA:-} -c fm_v_$name.hip \
    -o build/v_$name/$tgt.o --save-temps 2>/dev/null
python3 - fm_v_$name <<'PY'
import re, sys
s = open(sys.argv[1] + '-hip-amdgcn-amd-amdhsa-gfx950.s').read()
for blk in s.split('  - .agpr_count')[1:]:
    n = re.search(r'\.name:\s+(\S+)', blk).group(1)
    if 'k_matchILb0' in n or 'k_emitILb0' in n or 'k_encode' in n or 'k_treeILb0' in n:
        print(sys.argv[1], 'vgpr', re.search(r'\.vgpr_count:\s+(\d+)', blk).group(1), 'spill', re.search(r'\.vgpr_spill_count:\s+(\d+)', blk).group(1))
PY
rm -f fm_v_$name*
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/libfcx_$name.so build/v_$name/$tgt.o $(ls build/*.o | grep -v $tgt.o) \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf build/v_$name ../lib/libfcx.so.[0-9]*
