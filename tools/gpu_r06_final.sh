# Round-6 final GPU pass: the whole -m gpu suite, smoke, the default bench line, then the rocprofv3
# kernel stats and PMC traffic passes per leg (tools/gpu_r06_prof.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r06_full.sh && bash tools/gpu_r06_prof.sh
