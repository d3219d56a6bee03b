set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/dbg/qa_o_dbg.py > gpurun_out/r5ad_dbg.log 2>&1; rc=$?
cat gpurun_out/r5ad_dbg.log | grep -v amdgpu.ids | tail -40
exit $rc
