# parity (golden cases, mosaics, forced tile modes) + every full-size digest leg with its stage times
# (tools/devbench.py); summary: bash tools/gpu_check_summary.sh
set -u
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m "gpu and not slow" > gpurun_out/gs_parity.log 2>&1 || exit 1
timeout -k 10 200 python tools/devbench.py --kind rand --seed 4 --mib 1024 --check hl_rand_1GiB > gpurun_out/gs_rand.log 2>&1 || exit 1
timeout -k 10 200 python tools/devbench.py --kind rand --seed 2 --mib 64 --block 65536 --check cfg2_rand_64MiB > gpurun_out/gs_c2.log 2>&1 || exit 1
timeout -k 10 200 python tools/devbench.py --kind text --seed 3 --mib 1024 --check hl_text_1GiB > gpurun_out/gs_text.log 2>&1 || exit 1
timeout -k 10 200 python tools/devbench.py --kind text --seed 3 --mib 1024 --block 262144 --check cfg3_text_1GiB > gpurun_out/gs_c3.log 2>&1 || exit 1
timeout -k 10 200 python tools/devbench.py --kind runs --seed 5 --mib 1024 --check cfg5b_runs_1GiB > gpurun_out/gs_runs.log 2>&1 || exit 1
timeout -k 10 200 python tools/devbench.py --kind zeros --seed 0 --mib 1024 --check cfg5a_zeros_1GiB > gpurun_out/gs_zeros.log 2>&1 || exit 1
timeout -k 10 200 python tools/devbench.py --kind dna --seed 6 --mib 1024 > gpurun_out/gs_dna.log 2>&1 || exit 1
