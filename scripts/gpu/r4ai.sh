# Round 4: decode split-K granules for up to 4 slices (polled together): tests, TP=1 step, 70B TP=8 rank bench, AWQ down sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "splitk or awq or decode_gemm or norm" tests/test_streamk_gpu.py tests/test_fused_ar_gpu.py > gpurun_out/r4ai_tests.log 2>&1 || { tail -40 gpurun_out/r4ai_tests.log; exit 1; }
tail -1 gpurun_out/r4ai_tests.log
timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only > gpurun_out/r4ai_step.log 2>&1 || { tail -20 gpurun_out/r4ai_step.log; exit 1; }
grep '^{' gpurun_out/r4ai_step.log
timeout -k 10 400 python -u benchmarks/tp_rank_bench.py > gpurun_out/r4ai_tp8.log 2>&1 || { tail -30 gpurun_out/r4ai_tp8.log; exit 1; }
grep '^{' gpurun_out/r4ai_tp8.log | cut -c1-700
timeout -k 10 500 python -u benchmarks/tp_rank_bench.py --sweep --kinds qkv,down --iters 30 > gpurun_out/r4ai_tp8_sweep.log 2>&1 || { tail -30 gpurun_out/r4ai_tp8_sweep.log; exit 1; }
grep '"kind"\|best' gpurun_out/r4ai_tp8_sweep.log | cut -c1-300
timeout -k 10 600 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --quantization awq --kinds down > gpurun_out/r4ai_awq_down.log 2>&1 || { tail -30 gpurun_out/r4ai_awq_down.log; exit 1; }
grep '^{' gpurun_out/r4ai_awq_down.log | cut -c1-200
