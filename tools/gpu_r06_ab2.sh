set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
NO_TRANS=1 SETS="${SETS:-rand text|cur:0 e7:0 e72:0 e72b:0}" bash tools/gpu_r06_ab.sh
