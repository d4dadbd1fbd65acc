# Development: phase-timing variants of libfcx.so, each with one of k_match's timing exits compiled
# into the product kernel (FCX_MATCH_EXIT), as my_compress_amd/lib/libfcx_x<bit>.so; time them with
# VARS="x16 x4096 ..." bash tools/gpu_ab.sh (the output of such a library is invalid).
set -eu
cd "$(dirname "$0")/../my_compress_amd/csrc"
make -s
for bit in ${BITS:-16 4096 32 64 256}; do
  mkdir -p build/x$bit
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I../../include -I. \
      -DFCX_MATCH_EXIT=${bit}u -c fcx_match.hip -o build/x$bit/fcx_match.o
  objs=$(ls build/*.o | grep -v fcx_match.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/libfcx_x$bit.so build/x$bit/fcx_match.o $objs \
      -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
