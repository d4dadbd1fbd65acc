# A/B of the pipelined launch (fcx_ctx_set_groups) on the 1 GiB legs, digests checked
set -u
G="${GROUPS_LIST:-1,2,4,8}"
timeout -k 10 240 python tools/devbench.py --kind rand --seed 4 --mib 1024 --reps 5 --groups $G --check hl_rand_1GiB > gpurun_out/grp_rand.log 2>&1 || exit 1
timeout -k 10 240 python tools/devbench.py --kind text --seed 3 --mib 1024 --reps 5 --groups $G --check hl_text_1GiB > gpurun_out/grp_text.log 2>&1 || exit 1
timeout -k 10 240 python tools/devbench.py --kind runs --seed 5 --mib 1024 --reps 3 --groups $G --check cfg5b_runs_1GiB > gpurun_out/grp_runs.log 2>&1 || exit 1
for m in 128 256 512; do
  timeout -k 10 240 python tools/devbench.py --kind rand --seed 4 --mib $m --reps 5 --groups $G > gpurun_out/grp_rand_$m.log 2>&1 || exit 1
  timeout -k 10 240 python tools/devbench.py --kind text --seed 3 --mib $m --reps 5 --groups $G > gpurun_out/grp_text_$m.log 2>&1 || exit 1
done
