# quick GPU check: compress parity tests (not slow) + 1 GiB legs with digests (devbench)
set -u
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m "gpu and not slow" --timeout 500 --timeout-method thread > gpurun_out/tq.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/tq.log; [ $rc -eq 0 ] || exit 1
for leg in ${LEGS:-runs:5:cfg5b_runs_1GiB rand:4:hl_rand_1GiB text:3:hl_text_1GiB zeros:0:cfg5a_zeros_1GiB}; do
  IFS=: read kind seed chk <<< "$leg"
  timeout -k 10 240 python tools/devbench.py --kind $kind --seed $seed --mib 1024 --reps 5 --groups 1 --check $chk > gpurun_out/dq_$kind.log 2>&1 || exit 1
done
