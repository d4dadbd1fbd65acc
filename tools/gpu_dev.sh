# development loop: fast GPU parity (golden, forced modes, dna, mosaics, edges), then
# per-stage timing + digest of the 1 GiB legs named in $LEGS (kind:seed:check)
set -u
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m "gpu and not slow" tests/test_gpu_parity.py > gpurun_out/tdev.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/tdev.log; [ $rc -eq 0 ] || exit 1
for leg in ${LEGS:-rand:4:hl_rand_1GiB text:3:hl_text_1GiB dna:6:-}; do
  IFS=: read kind seed check <<< "$leg"
  c=""; [ "$check" != "-" ] && c="--check $check"
  timeout -k 10 300 python tools/devbench.py --kind $kind --seed $seed --mib 1024 $c > gpurun_out/dev_$kind.log 2>&1 || exit 1
done
