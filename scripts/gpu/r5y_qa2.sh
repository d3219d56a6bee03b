# Round 5: fused QKV + attention with split-K GEMMs (tests), 70B TP8 rank qkv sweep with the fused launch
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "qkv_attention_fused or qkv_rope or attention or decode" > gpurun_out/r5y_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5y_tests.log; exit 1; }
tail -2 gpurun_out/r5y_tests.log
timeout -k 10 300 python -u -m pytest tests/test_fused_ar_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5y_far.log 2>&1 || { echo F_FAIL; tail -30 gpurun_out/r5y_far.log; exit 1; }
tail -1 gpurun_out/r5y_far.log
timeout -k 10 600 python -u benchmarks/tp_rank_bench.py --sweep --kinds qkv --iters 30 > gpurun_out/r5y_tp8.log 2>&1 || { tail -30 gpurun_out/r5y_tp8.log; exit 1; }
grep '^{' gpurun_out/r5y_tp8.log | cut -c1-250
