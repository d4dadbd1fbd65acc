set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_dist_rehearsal.sh && for f in reh_n1_fcx reh_n1_torch reh_n2_gloo; do echo "== $f"; tail -c 700 gpurun_out/$f.json; echo; done
