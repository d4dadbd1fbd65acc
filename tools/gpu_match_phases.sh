# k_match phase times: the kernel alone (fcx_debug_match, nothing downstream runs) from the
# FCX_MATCH_EXIT libraries of tools/phase_libs.sh (lib/libfcx_x<bit>.so) and the product library
set -u
for kind in ${KINDS:-text rand}; do
  timeout -k 10 200 python tools/matchab.py --kind $kind --mib 1024 --reps 3 0 > gpurun_out/mp_${kind}_A.log 2>&1 || exit 1
  for bit in ${BITS:-16 4096 32 64 256}; do
    FCX_LIB=$PWD/my_compress_amd/lib/libfcx_x$bit.so timeout -k 10 200 python tools/matchab.py --kind $kind --mib 1024 --reps 3 0 > gpurun_out/mp_${kind}_x$bit.log 2>&1 || exit 1
  done
done
