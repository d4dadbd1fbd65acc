# second half of the round-end evidence (after tools/gpu_ckpt.sh): N=2 rehearsal (two ranks on one
# GPU over gloo), rocprofv3 kernel stats of the default command with every leg, PMC traffic per leg
set -u
R=$PWD
FCX_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --no-text --no-decode > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || exit 1
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_all -o run --output-format csv -- python3 $R/bench.py --no-lz78 > $R/gpurun_out/prof_all.json 2> $R/gpurun_out/prof_all.err) || exit 1
LEGS="${LEGS:-rand:rand:1048576 text:text:1048576 c3:text:262144 zeros:zeros:1048576 runs:runs:1048576}" bash tools/pmc_traffic.sh || exit 1
