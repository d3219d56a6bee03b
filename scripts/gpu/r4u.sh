# Round 4: fused row-parallel GEMM + all-reduce (epilogue_ar): kernel tests, TP = 2 engine tests,
# 70B TP = 8 rank bench with the fused exchange against a loopback region, and the TP = 1 step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_ar_gpu.py > gpurun_out/r4u_fused_tests.log 2>&1 || { tail -40 gpurun_out/r4u_fused_tests.log; exit 1; }
tail -3 gpurun_out/r4u_fused_tests.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tp_gpu.py > gpurun_out/r4u_tp_tests.log 2>&1 || { tail -40 gpurun_out/r4u_tp_tests.log; exit 1; }
tail -3 gpurun_out/r4u_tp_tests.log
timeout -k 10 400 python -u benchmarks/tp_rank_bench.py > gpurun_out/r4u_tp8_stub.log 2>&1 || { tail -30 gpurun_out/r4u_tp8_stub.log; exit 1; }
grep '^{' gpurun_out/r4u_tp8_stub.log
timeout -k 10 400 python -u benchmarks/tp_rank_bench.py --fused-ar > gpurun_out/r4u_tp8_fused.log 2>&1 || { tail -30 gpurun_out/r4u_tp8_fused.log; exit 1; }
grep '^{' gpurun_out/r4u_tp8_fused.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r4u_timeline.log 2>&1 || { tail -30 gpurun_out/r4u_timeline.log; exit 1; }
head -3 gpurun_out/r4u_timeline.log
