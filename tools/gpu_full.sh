# full GPU validation: every gpu test (incl. GiB digests), then an N=2 bench rehearsal
set -u
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/tfull.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/tfull.log; [ $rc -eq 0 ] || exit 1
FCX_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --mib 256 --dist-backend gloo --no-text > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err; echo "n2 rc=$?" >> gpurun_out/bench_n2.err
