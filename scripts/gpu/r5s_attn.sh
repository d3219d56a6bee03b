# Round 5: decode rows in the flash prefill launch (one attention launch per prefill / mixed step)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r5s_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5s_tests.log; exit 1; }
tail -2 gpurun_out/r5s_tests.log
timeout -k 10 300 python -u benchmarks/timeline.py --prefill --batch 8 --ctx 50 > gpurun_out/r5s_prefill_timeline.log 2>&1 || { tail -30 gpurun_out/r5s_prefill_timeline.log; exit 1; }
grep -h '"step_us"' gpurun_out/r5s_prefill_timeline.log | cut -c1-120
timeout -k 10 300 python -u benchmarks/timeline.py --mixed 48 --batch 8 --ctx 100 > gpurun_out/r5s_mixed_timeline.log 2>&1 || { tail -30 gpurun_out/r5s_mixed_timeline.log; exit 1; }
grep -h '"step_us"' gpurun_out/r5s_mixed_timeline.log | cut -c1-120
