set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
t0=$(date +%s)
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=12 > gpurun_out/r5al_tier.log 2>&1; rc=$?
echo "gpu tier wall s: $(( $(date +%s) - t0 ))" | tee -a gpurun_out/r5al_tier.log
grep -A 14 "slowest" gpurun_out/r5al_tier.log | head -16
tail -2 gpurun_out/r5al_tier.log
exit $rc
