# round-3 profiles: rocprofv3 kernel stats (main leg; every leg), PMC traffic passes per leg,
# and the single-GPU strong-scaling predictor (tools/shardscale.py) for rand and text
set -u
R=$PWD
timeout -k 10 300 python tools/shardscale.py --kind rand --seed 4 --out gpurun_out/shardscale_rand.json > gpurun_out/shardscale_rand.log 2>&1 || exit 1
timeout -k 10 300 python tools/shardscale.py --kind text --seed 3 --out gpurun_out/shardscale_text.json > gpurun_out/shardscale_text.log 2>&1 || exit 1
timeout -k 10 200 python tools/matchphase.py --kind text --seed 3 --mib 256 > gpurun_out/phase_text.log 2>&1 || exit 1
timeout -k 10 200 python tools/matchphase.py --kind rand --seed 4 --mib 256 > gpurun_out/phase_rand.log 2>&1 || exit 1
bash tools/gpu_prof_round.sh
