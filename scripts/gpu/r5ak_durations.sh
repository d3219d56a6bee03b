set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=40 > gpurun_out/r5ak_dur.log 2>&1; rc=$?
grep -A 45 "slowest" gpurun_out/r5ak_dur.log | head -50
tail -1 gpurun_out/r5ak_dur.log
exit $rc
