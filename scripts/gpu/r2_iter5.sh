set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_custom_allreduce_gpu.py tests/test_tp_gpu.py -x -v --timeout 280 --timeout-method thread > gpurun_out/r2_tp5.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/r2_tp5.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r2_tp5.log | tail -12
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2_gpu_all5.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/r2_gpu_all5.log; exit 1; }
tail -2 gpurun_out/r2_gpu_all5.log
