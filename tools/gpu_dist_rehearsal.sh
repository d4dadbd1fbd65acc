# N=1 rehearsal of the multi-rank bench path over nccl (RCCL): C++ fcx_dist concat (gather,
# all-gather) and torch P2P, main + weak legs, digests checked
set -u
for impl in fcx torch; do
  for mode in gather allgather; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --dist-rehearsal --steps 3 --warmup 1 --no-text --no-decode --no-cpu-baseline --no-host-path --concat $mode --concat-impl $impl > gpurun_out/reh_${impl}_$mode.json 2> gpurun_out/reh_${impl}_$mode.err || exit 1
  done
done
