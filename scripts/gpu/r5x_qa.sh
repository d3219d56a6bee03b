# Round 5: fused QKV projection + decode attention launch: kernel tests, engine parity, decode timeline, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "qkv_attention_fused or qkv_rope or attention" > gpurun_out/r5x_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5x_tests.log; exit 1; }
tail -3 gpurun_out/r5x_tests.log
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5x_engine.log 2>&1 || { echo E_FAIL; tail -60 gpurun_out/r5x_engine.log; exit 1; }
tail -2 gpurun_out/r5x_engine.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r5x_timeline.log 2>&1 || { tail -30 gpurun_out/r5x_timeline.log; exit 1; }
head -c 600 gpurun_out/r5x_timeline.log | tail -c 500
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5x_bench.log 2>&1 || { tail -30 gpurun_out/r5x_bench.log; exit 1; }
tail -1 gpurun_out/r5x_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','max_gpu_step_ms','timed_engine_idle_ms')})"
