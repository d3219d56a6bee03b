# Round 5: GPU tier (new sampler test: alternating batch sizes) + driver bench with wave breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "sample" --timeout 120 --timeout-method thread > gpurun_out/r5c_sampler.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5c_sampler.log; exit 1; }
tail -2 gpurun_out/r5c_sampler.log
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r5c_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5c_tests.log; exit 1; }
tail -2 gpurun_out/r5c_tests.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5c_bench.log 2>&1 || { tail -30 gpurun_out/r5c_bench.log; exit 1; }
tail -1 gpurun_out/r5c_bench.log | cut -c1-1500
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r5c_bench_awq.log 2>&1 || { tail -30 gpurun_out/r5c_bench_awq.log; exit 1; }
tail -1 gpurun_out/r5c_bench_awq.log | cut -c1-600
