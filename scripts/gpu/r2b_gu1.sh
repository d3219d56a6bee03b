set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm_silu" --timeout 120 --timeout-method thread > gpurun_out/r2b_gu_tests.log 2>&1 || { echo T_FAIL; tail -40 gpurun_out/r2b_gu_tests.log; exit 1; }
tail -1 gpurun_out/r2b_gu_tests.log
timeout -k 10 500 python -u benchmarks/decode_sweep.py --kinds gate_up --ctx 100 > gpurun_out/r2b_gu_sweep.log 2>&1 || { tail -30 gpurun_out/r2b_gu_sweep.log; exit 1; }
grep "^{" gpurun_out/r2b_gu_sweep.log
