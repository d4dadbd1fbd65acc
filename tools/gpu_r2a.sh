# round-2 check: new parity tests (fast), bench N=1 (no extra legs), N=2 gloo rehearsal
set -u
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 -m "gpu and not slow" tests/test_gpu_parity.py tests/test_gpu_decode.py > gpurun_out/t2a.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t2a.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-lz78 --legs dna > gpurun_out/b2a_n1.json 2> gpurun_out/b2a_n1.err || exit 1
FCX_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --no-text --no-decode > gpurun_out/b2a_n2.json 2> gpurun_out/b2a_n2.err || exit 1
