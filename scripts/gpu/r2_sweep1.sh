set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or awq" > gpurun_out/r2_kern1.log 2>&1 || { echo KERNTEST_FAIL; tail -30 gpurun_out/r2_kern1.log; exit 1; }
tail -3 gpurun_out/r2_kern1.log
timeout -k 10 500 python -u benchmarks/decode_sweep.py --iters 50 > gpurun_out/r2_sweep1.log 2>&1
rc=$?; tail -5 gpurun_out/r2_sweep1.log; exit $rc
