# Round 5: bf16 register-stationary decode GEMM sweep (vs the tile kernels), int4 kx tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "awq" > gpurun_out/r5o_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5o_tests.log; exit 1; }
tail -2 gpurun_out/r5o_tests.log
timeout -k 10 400 python -u benchmarks/dense_kx_sweep.py > gpurun_out/r5o_sweep.log 2>&1 || { tail -30 gpurun_out/r5o_sweep.log; exit 1; }
echo sweep_ok
