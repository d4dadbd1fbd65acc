set -u
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --dist-rehearsal --steps 3 --warmup 1 --no-text --no-decode --no-cpu-baseline --no-host-path > gpurun_out/g2_reh1.json 2> gpurun_out/g2_reh1.err || exit 1
FCX_BENCH_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 bench.py --dist-backend gloo --steps 2 --warmup 1 --no-text --no-decode --no-cpu-baseline --no-host-path > gpurun_out/g2_reh2.json 2> gpurun_out/g2_reh2.err || exit 1
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --no-host-path --no-lz78 > gpurun_out/g3_bench.json 2> gpurun_out/g3_bench.err || exit 1
