set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/r2b_attn_tests.log 2>&1 || { echo T_FAIL; tail -40 gpurun_out/r2b_attn_tests.log; exit 1; }
tail -2 gpurun_out/r2b_attn_tests.log
timeout -k 10 200 python -u benchmarks/attn_phases.py > gpurun_out/r2b_attn_phases.log 2>&1 || { tail -30 gpurun_out/r2b_attn_phases.log; exit 1; }
cat gpurun_out/r2b_attn_phases.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r2b_timeline2.log 2>&1 || { tail -30 gpurun_out/r2b_timeline2.log; exit 1; }
grep -v "^{\"kernel\"" gpurun_out/r2b_timeline2.log | cut -c1-600 | tail -3
grep "attention" gpurun_out/r2b_timeline2.log | head -3
