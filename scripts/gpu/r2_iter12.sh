set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 200 --timeout-method thread > gpurun_out/r2_kern12.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/r2_kern12.log; exit 1; }
tail -1 gpurun_out/r2_kern12.log
timeout -k 10 200 python -u benchmarks/attn_phases.py > gpurun_out/r2_attn_phases12.log 2>&1 || { tail -20 gpurun_out/r2_attn_phases12.log; exit 1; }
grep ctx gpurun_out/r2_attn_phases12.log
timeout -k 10 300 python -u benchmarks/micro_gpu.py --only attn > gpurun_out/r2_attn12.log 2>&1 || { tail -20 gpurun_out/r2_attn12.log; exit 1; }
grep attention gpurun_out/r2_attn12.log
