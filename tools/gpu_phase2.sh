# k_match phase timing (fcx_debug_match exits) + devbench legs
set -u
for k in ${PH_KINDS:-runs:5 rand:4}; do
  IFS=: read kind seed <<< "$k"
  timeout -k 10 200 python tools/matchphase.py --kind $kind --seed $seed --mib 256 > gpurun_out/ph_$kind.log 2>&1 || exit 1
done
for leg in ${LEGS:-rand:4:hl_rand_1GiB runs:5:cfg5b_runs_1GiB}; do
  IFS=: read kind seed chk <<< "$leg"
  timeout -k 10 240 python tools/devbench.py --kind $kind --seed $seed --mib 1024 --reps 5 --groups 1 --check $chk > gpurun_out/dq_$kind.log 2>&1 || exit 1
done
