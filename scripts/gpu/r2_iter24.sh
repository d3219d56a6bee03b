set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "sample" --timeout 120 --timeout-method thread > gpurun_out/r2_s24.log 2>&1 || { echo S_FAIL; tail -60 gpurun_out/r2_s24.log; exit 1; }
tail -3 gpurun_out/r2_s24.log
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2_gpu24.log 2>&1 || { echo GPU_FAIL; tail -40 gpurun_out/r2_gpu24.log; exit 1; }
tail -2 gpurun_out/r2_gpu24.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2_bench24.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/r2_bench24.log; exit 1; }
tail -1 gpurun_out/r2_bench24.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','timed_eager_steps','timed_graph_captures')})"
