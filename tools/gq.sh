# quick check of a k_match change: non-slow parity tests, then k_match phase timings and full-size digests
set -u
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m "gpu and not slow" > gpurun_out/gq_parity.log 2>&1 || exit 1
timeout -k 10 200 python tools/matchab.py --kind text --mib 256 --reps 3 0 0x20 0x40 1 0x400000 > gpurun_out/gq_text.log 2>&1 || exit 1
timeout -k 10 200 python tools/matchab.py --kind dna --mib 256 --reps 3 0 > gpurun_out/gq_dna.log 2>&1 || exit 1
timeout -k 10 200 python tools/devbench.py --kind text --seed 3 --mib 1024 --check hl_text_1GiB > gpurun_out/gq_bq_text.log 2>&1 || exit 1
timeout -k 10 200 python tools/devbench.py --kind rand --seed 4 --mib 1024 --check hl_rand_1GiB > gpurun_out/gq_bq_rand.log 2>&1 || exit 1
