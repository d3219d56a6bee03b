# Round 3: flash prefill kernel v4 + TP tests (two-shot at 600 tokens, peer-stop timeout path)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu/r3_flash4.sh || exit 1
timeout -k 10 700 python -u -m pytest tests/test_tp_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r3_tp1_tests.log 2>&1 || { tail -60 gpurun_out/r3_tp1_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r3_tp1_tests.log | tail -6
