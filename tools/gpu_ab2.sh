# A/B of lib/libfcx.so vs $ALT on rand/text at 1 GiB and 128 MiB (the N=8 per-rank shard), + quick parity
set -u
ALT=${ALT:-my_compress_amd/lib/libfcx_v.so}
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q -m "gpu and not slow" > gpurun_out/tq.log 2>&1 || exit 1
for kind in ${KINDS:-rand text}; do
  case $kind in text) seed=3;; rand) seed=4;; runs) seed=5;; dna) seed=6;; *) seed=0;; esac
  for mib in ${MIBS:-1024 128}; do
    timeout -k 10 200 python tools/devbench.py --kind $kind --seed $seed --mib $mib > gpurun_out/ab_a_${kind}_$mib.log 2>&1 || exit 1
    FCX_LIB=$PWD/$ALT timeout -k 10 200 python tools/devbench.py --kind $kind --seed $seed --mib $mib > gpurun_out/ab_b_${kind}_$mib.log 2>&1 || exit 1
  done
done
