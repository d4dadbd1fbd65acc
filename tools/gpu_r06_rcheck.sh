set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/r06_rcheck.py > gpurun_out/r06_rcheck.log 2>&1; rc=$?; cat gpurun_out/r06_rcheck.log | grep -v amdgpu.ids; exit $rc
