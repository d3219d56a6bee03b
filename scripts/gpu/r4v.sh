# Round 4: fused row-parallel GEMM + all-reduce v2 (no system-scope fences: ordered sc0 sc1 stores / loads)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_ar_gpu.py > gpurun_out/r4v_fused_tests.log 2>&1 || { tail -40 gpurun_out/r4v_fused_tests.log; exit 1; }
tail -3 gpurun_out/r4v_fused_tests.log
timeout -k 10 400 python -u benchmarks/tp_rank_bench.py --fused-ar > gpurun_out/r4v_tp8_fused.log 2>&1 || { tail -30 gpurun_out/r4v_tp8_fused.log; exit 1; }
grep '^{' gpurun_out/r4v_tp8_fused.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tp_gpu.py > gpurun_out/r4v_tp_tests.log 2>&1 || { tail -40 gpurun_out/r4v_tp_tests.log; exit 1; }
tail -3 gpurun_out/r4v_tp_tests.log
