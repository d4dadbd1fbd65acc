# full GPU validation: every gpu test (incl. the GiB digests and config-4 rank segments),
# the default bench line, an N=2 rehearsal (two ranks on one GPU over gloo)
set -u
timeout -k 10 1500 python -u -m pytest tests -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/tfull.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/tfull.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || exit 1
FCX_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --no-text --no-decode > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err; echo "n2 rc=$?" >> gpurun_out/bench_n2.err
