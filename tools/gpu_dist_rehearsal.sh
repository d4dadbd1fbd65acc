# Rehearsals of the multi-rank bench path on one GPU: N=1 over nccl (RCCL) through the C++
# pipelined gather (fcx_dist_compress_gather) and the torch P2P form, and N=2 over gloo with both
# ranks on cuda:0 (the gather-aware split and the sub-batch protocol), digests checked
set -u
for impl in fcx torch; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --dist-rehearsal --steps 3 --warmup 1 --no-text --no-decode --no-cpu-baseline --no-host-path --concat pipe --concat-impl $impl > gpurun_out/reh_n1_$impl.json 2> gpurun_out/reh_n1_$impl.err || exit 1
done
FCX_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 bench.py --dist-backend gloo --steps 2 --warmup 1 --no-text --no-decode --no-host-path --concat pipe > gpurun_out/reh_n2_gloo.json 2> gpurun_out/reh_n2_gloo.err || exit 1
