set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "sample or graph_equals or async" > gpurun_out/r6f_t.log 2>&1 || { tail -30 gpurun_out/r6f_t.log; exit 1; }
tail -1 gpurun_out/r6f_t.log
bash scripts/gpu/run.sh r6f timeline bench2
