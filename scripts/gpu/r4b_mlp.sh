# Round 4: fused decode MLP — kernel numerics, engine parity (graph == eager == fp32), decode-step timeline, driver bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_mlp_fused_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4b_mlp_test.log 2>&1 || { echo MLP_TEST_FAIL; tail -60 gpurun_out/r4b_mlp_test.log; exit 1; }
tail -3 gpurun_out/r4b_mlp_test.log
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4b_engine_test.log 2>&1 || { echo ENGINE_TEST_FAIL; tail -60 gpurun_out/r4b_engine_test.log; exit 1; }
tail -3 gpurun_out/r4b_engine_test.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r4b_timeline.log 2>&1 || { tail -30 gpurun_out/r4b_timeline.log; exit 1; }
grep '"launches"' gpurun_out/r4b_timeline.log | cut -c1-1500
VGATE_FUSED_MLP=0 timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r4b_timeline_unfused.log 2>&1 || { tail -30 gpurun_out/r4b_timeline_unfused.log; exit 1; }
grep '"launches"' gpurun_out/r4b_timeline_unfused.log | cut -c1-300
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4b_bench.log 2>&1 || { tail -30 gpurun_out/r4b_bench.log; exit 1; }
tail -1 gpurun_out/r4b_bench.log | cut -c1-700
