set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "sample or prefill_lds" > gpurun_out/r2_kern3.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/r2_kern3.log; exit 1; }
tail -2 gpurun_out/r2_kern3.log
timeout -k 10 300 python -u benchmarks/sampler_stress.py --groups 40 > gpurun_out/r2_sampler_stress2.log 2>&1 || { tail -20 gpurun_out/r2_sampler_stress2.log; exit 1; }
grep -v amdgpu gpurun_out/r2_sampler_stress2.log | grep -v sampler_stress
timeout -k 10 400 python -u benchmarks/prefill_gemm_bench.py > gpurun_out/r2_prefill_gemm1.log 2>&1 || { tail -20 gpurun_out/r2_prefill_gemm1.log; exit 1; }
grep -v amdgpu gpurun_out/r2_prefill_gemm1.log
timeout -k 10 200 python -u benchmarks/timeline.py --json gpurun_out/r2_timeline2.json > gpurun_out/r2_timeline2.log 2>&1 && head -1 gpurun_out/r2_timeline2.log
