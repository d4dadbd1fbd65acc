# round-end profiles on one GPU (the part of gpu_round.sh after gpu_full.sh): rocprofv3
# kernel stats of the main leg alone (its k_match average is the roofline kernel's time) and
# of the default command with every leg, then PMC traffic passes for every leg
set -u
R=$PWD
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_n1 -o run --output-format csv -- python3 $R/bench.py --no-text --no-decode --no-host-path > $R/gpurun_out/prof_n1.json 2> $R/gpurun_out/prof_n1.err) || exit 1
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_all -o run --output-format csv -- python3 $R/bench.py --no-lz78 > $R/gpurun_out/prof_all.json 2> $R/gpurun_out/prof_all.err) || exit 1
LEGS="${LEGS:-rand:rand:1048576 text:text:1048576 c3:text:262144 zeros:zeros:1048576 runs:runs:1048576 dna:dna:1048576}" bash tools/pmc_traffic.sh || exit 1
