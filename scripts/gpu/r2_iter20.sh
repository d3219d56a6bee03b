set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "attention_prefill_long" --timeout 120 --timeout-method thread > gpurun_out/r2_long20.log 2>&1 || { echo LONG_FAIL; tail -40 gpurun_out/r2_long20.log; exit 1; }
tail -3 gpurun_out/r2_long20.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2_gpu20.log 2>&1 || { echo GPU_FAIL; tail -40 gpurun_out/r2_gpu20.log; exit 1; }
tail -3 gpurun_out/r2_gpu20.log
