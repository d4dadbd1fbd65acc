# Round-6 profiles on one GPU: rocprofv3 kernel stats of bench.py per leg, then the PMC HBM traffic
# passes (FETCH_SIZE, WRITE_SIZE) per 1 GiB leg.  Summaries: python tools/pmc_traffic.py r06;
# python tools/roofline_check.py r06 (after copying the stats into profiles/).
set -u
LEGS="${LEGS:-rand:rand:1048576:1024 c2:rand:65536:64 text:text:1048576:1024 c3:text:262144:1024 zeros:zeros:1048576:1024 runs:runs:1048576:1024 dna:dna:1048576:1024 mix:mix:1048576:1024}" SKIP_SQ=1 bash tools/gpu_prof_round.sh
