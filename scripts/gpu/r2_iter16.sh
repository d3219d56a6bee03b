set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "awq or silu or prefill" --timeout 200 --timeout-method thread > gpurun_out/r2_kern16.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/r2_kern16.log; exit 1; }
tail -1 gpurun_out/r2_kern16.log
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2_eng16.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/r2_eng16.log; exit 1; }
tail -1 gpurun_out/r2_eng16.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r2_bench16_awq.json.log 2>&1 || { tail -20 gpurun_out/r2_bench16_awq.json.log; exit 1; }
tail -1 gpurun_out/r2_bench16_awq.json.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench16_bf16.json.log 2>&1 || { tail -20 gpurun_out/r2_bench16_bf16.json.log; exit 1; }
tail -1 gpurun_out/r2_bench16_bf16.json.log
