# Round 5: bf16 gate_up on the register-stationary kernel (decode plan): kernel tests, bf16 timeline, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "kx or awq or gemm" > gpurun_out/r5p_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5p_tests.log; exit 1; }
tail -2 gpurun_out/r5p_tests.log
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r5p_engine.log 2>&1 || { echo E_FAIL; tail -60 gpurun_out/r5p_engine.log; exit 1; }
tail -2 gpurun_out/r5p_engine.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r5p_timeline_bf16.log 2>&1 || { tail -30 gpurun_out/r5p_timeline_bf16.log; exit 1; }
grep -h '"step_us"' gpurun_out/r5p_timeline_bf16.log | cut -c1-100
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5p_bench.log 2>&1 || { tail -30 gpurun_out/r5p_bench.log; exit 1; }
tail -1 gpurun_out/r5p_bench.log | cut -c1-300
