# k_emit path timing (development exits, tools/emitab.py) on rand and text, plus parity of the current library
set -u
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m "gpu and not slow" > gpurun_out/ge_parity.log 2>&1 || exit 1
timeout -k 10 200 python tools/devbench.py --kind rand --seed 4 --mib 1024 --check hl_rand_1GiB > gpurun_out/ge_rand.log 2>&1 || exit 1
timeout -k 10 200 python tools/emitab.py --kind rand 0 1 2 3 4 8 > gpurun_out/ge_emit_rand.log 2>&1 || exit 1
timeout -k 10 200 python tools/emitab.py --kind text 0 2 4 8 > gpurun_out/ge_emit_text.log 2>&1 || exit 1
