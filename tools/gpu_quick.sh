# quick GPU check used during development: parity tests + rand/text timing
set -u
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q -m "gpu and not slow" > gpurun_out/tq.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/tq.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/devbench.py --kind rand --seed 4 --mib 1024 --check hl_rand_1GiB > gpurun_out/bq_rand.log 2>&1 || exit 1
timeout -k 10 200 python tools/devbench.py --kind text --seed 3 --mib 1024 --check hl_text_1GiB > gpurun_out/bq_text.log 2>&1 || exit 1
for extra in "$@"; do eval "$extra" || exit 1; done
