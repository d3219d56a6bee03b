# Round 5: register-stationary int4 decode kernel (gemm_awq_kx.hip): numerics, AWQ engine parity, timeline, AWQ bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "awq" > gpurun_out/r5j_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5j_tests.log; exit 1; }
tail -2 gpurun_out/r5j_tests.log
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "awq or AWQ" > gpurun_out/r5j_engine.log 2>&1 || { echo E_FAIL; tail -60 gpurun_out/r5j_engine.log; exit 1; }
tail -2 gpurun_out/r5j_engine.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 --quantization awq > gpurun_out/r5j_timeline.log 2>&1 || { tail -30 gpurun_out/r5j_timeline.log; exit 1; }
grep '"step_us"' gpurun_out/r5j_timeline.log | cut -c1-300
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r5j_bench_awq.log 2>&1 || { tail -30 gpurun_out/r5j_bench_awq.log; exit 1; }
tail -1 gpurun_out/r5j_bench_awq.log | cut -c1-400
