set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_tp_gpu.py -x -q --timeout 280 --timeout-method thread -k "half or per_8 or handoff or sample or graph_equals or async or tp2 or qwen" > gpurun_out/r6h_t.log 2>&1 || { tail -30 gpurun_out/r6h_t.log; exit 1; }
tail -1 gpurun_out/r6h_t.log
bash scripts/gpu/run.sh r6h py:benchmarks/probes/half_tile_probe.py timeline bench2
