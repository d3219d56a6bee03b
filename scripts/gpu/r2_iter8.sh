set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2_kern8.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/r2_kern8.log; exit 1; }
tail -2 gpurun_out/r2_kern8.log
timeout -k 10 300 python -u benchmarks/decode_sweep.py --kinds gate_up > gpurun_out/r2_sweep8.log 2>&1 || { tail -20 gpurun_out/r2_sweep8.log; exit 1; }
grep '^{' gpurun_out/r2_sweep8.log | tail -8
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench8.json.log 2>&1 || { tail -20 gpurun_out/r2_bench8.json.log; exit 1; }
tail -1 gpurun_out/r2_bench8.json.log
