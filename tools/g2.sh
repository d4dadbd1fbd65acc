# round 4: text k_match phases + the pipelined gather (one-rank RCCL, two-rank gloo rehearsal)
set -u
timeout -k 10 200 python tools/matchab.py --kind text --mib 256 --reps 3 0 0x400000 0x100000 0x200000 0x20 0x40 1 > gpurun_out/g1_text.log 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dist.py > gpurun_out/g2_dist.log 2>&1 || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --dist-rehearsal --steps 3 --warmup 1 --no-text --no-decode --no-cpu-baseline --no-host-path > gpurun_out/g2_reh1.json 2> gpurun_out/g2_reh1.err || exit 1
FCX_BENCH_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 bench.py --dist-backend gloo --steps 2 --warmup 1 --no-text --no-decode --no-cpu-baseline --no-host-path > gpurun_out/g2_reh2.json 2> gpurun_out/g2_reh2.err || exit 1
timeout -k 10 200 python tools/matchab.py --kind rand --mib 256 --reps 3 0 0x20 0x1000 > gpurun_out/g1_rand.log 2>&1 || exit 1
