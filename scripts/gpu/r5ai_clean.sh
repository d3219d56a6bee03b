# Round 5: which GPU test leaves an in-launch hand-off word set (conftest fixture)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5ai_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5ai_tests.log | tail -15
grep -B2 -A2 "hand-off words left set" gpurun_out/r5ai_tests.log | head -30
exit 0
