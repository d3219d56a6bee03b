set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_kern2.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/r2_kern2.log; exit 1; }
tail -2 gpurun_out/r2_kern2.log
timeout -k 10 300 python -u benchmarks/sampler_stress.py --groups 100 > gpurun_out/r2_sampler_stress.log 2>&1 || { tail -20 gpurun_out/r2_sampler_stress.log; exit 1; }
cat gpurun_out/r2_sampler_stress.log | grep -v amdgpu
timeout -k 10 300 python -u benchmarks/decode_sweep.py --iters 100 --kinds qkv > gpurun_out/r2_sweep2.log 2>&1 || { tail -20 gpurun_out/r2_sweep2.log; exit 1; }
grep -v amdgpu gpurun_out/r2_sweep2.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench2.json.log 2>&1 || { tail -20 gpurun_out/r2_bench2.json.log; exit 1; }
tail -1 gpurun_out/r2_bench2.json.log
