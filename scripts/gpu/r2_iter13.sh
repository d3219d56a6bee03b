set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "awq or silu" --timeout 200 --timeout-method thread > gpurun_out/r2_kern13.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/r2_kern13.log; exit 1; }
tail -1 gpurun_out/r2_kern13.log
tail -1 gpurun_out/r2_kern13.log
timeout -k 10 300 python -u benchmarks/awq_sweep.py > gpurun_out/r2_awq_sweep13.log 2>&1 || { tail -20 gpurun_out/r2_awq_sweep13.log; exit 1; }
grep shape gpurun_out/r2_awq_sweep13.log
