# Round profiles on one GPU (run from the repo root under gpurun; outputs under gpurun_out/):
#   1. rocprofv3 kernel stats of bench.py per leg, one run each (prof_<leg>/run_kernel_stats.csv:
#      the leg's roofline kernel average = the bench line's kernel_ms), legs as name:kind:block:MiB
#   2. PMC HBM traffic passes per leg (tools/pmc_traffic.sh: FETCH_SIZE, WRITE_SIZE)
#   3. SQ counter sets A and B on the compress pipeline for text and rand (tools/pmc_match.sh)
# Summaries: python tools/pmc_traffic.py rNN; python tools/pmc_summary.py gpurun_out --json ...
set -u
R=$PWD
export TMPDIR=/tmp
LEGS="${LEGS:-rand:rand:1048576:1024 c2:rand:65536:64 text:text:1048576:1024 c3:text:262144:1024 zeros:zeros:1048576:1024 runs:runs:1048576:1024 dna:dna:1048576:1024}"
if [ -z "${SKIP_STATS:-}" ]; then
  for leg in $LEGS; do
    IFS=: read name kind block mib <<< "$leg"
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$name -o run --output-format csv -- python3 $R/bench.py --kind $kind --block $block --global-mib $mib --no-text --no-cpu-baseline --no-decode --no-host-path --no-lz78 --no-transition > $R/gpurun_out/prof_$name.json 2> $R/gpurun_out/prof_$name.err) || exit 1
  done
fi
if [ -z "${SKIP_TRAFFIC:-}" ]; then
  LEGS="$(for leg in $LEGS; do IFS=: read n k b m <<< "$leg"; [ "$m" = 1024 ] && echo -n "$n:$k:$b "; done)" bash tools/pmc_traffic.sh || exit 1
fi
if [ -z "${SKIP_SQ:-}" ]; then
  KINDS="${SQ_KINDS:-text rand}" bash tools/pmc_match.sh || exit 1
fi
