set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/dbg/flash_det.py > gpurun_out/r5aj_flash.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r5aj_flash.log | tail -45
exit $rc
