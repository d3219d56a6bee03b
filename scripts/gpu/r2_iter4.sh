set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_kern4.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/r2_kern4.log; exit 1; }
tail -2 gpurun_out/r2_kern4.log
timeout -k 10 300 python -u benchmarks/sampler_stress.py --groups 30 --nseg 32,64 > gpurun_out/r2_sampler_stress3.log 2>&1 || { tail -20 gpurun_out/r2_sampler_stress3.log; exit 1; }
grep -v amdgpu gpurun_out/r2_sampler_stress3.log | grep -v sampler_stress
timeout -k 10 400 python -u benchmarks/prefill_gemm_bench.py --ms 128,256,512,2048 > gpurun_out/r2_prefill_gemm2.log 2>&1 || { tail -20 gpurun_out/r2_prefill_gemm2.log; exit 1; }
grep -v amdgpu gpurun_out/r2_prefill_gemm2.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l)
    if 'summary' in d: print(d); continue
    print(d['model'],d['proj'],d['M'],d['ours_us'],d['hipblaslt_us'],d['ratio_vs_lib'])"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench4.json.log 2>&1 || { tail -20 gpurun_out/r2_bench4.json.log; exit 1; }
tail -1 gpurun_out/r2_bench4.json.log
