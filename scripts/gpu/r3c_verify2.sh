# Round 3 (session 3): re-check of the custom all-reduce timeout test, then TTFT (engine level) and the driver bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_tp_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r3c_tp.log 2>&1 || { echo TP_FAIL; tail -60 gpurun_out/r3c_tp.log; exit 1; }
tail -1 gpurun_out/r3c_tp.log
timeout -k 10 400 python -u benchmarks/ttft_probe.py --model Qwen/Qwen2.5-1.5B-Instruct --lens 512 2048 4096 --chunk 4096 > gpurun_out/r3c_ttft_qwen.log 2>&1 || { tail -30 gpurun_out/r3c_ttft_qwen.log; exit 1; }
grep '^{' gpurun_out/r3c_ttft_qwen.log
timeout -k 10 500 python -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 512 2048 4096 --chunk 4096 > gpurun_out/r3c_ttft_llama.log 2>&1 || { tail -30 gpurun_out/r3c_ttft_llama.log; exit 1; }
grep '^{' gpurun_out/r3c_ttft_llama.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3c_bench.log 2>&1 || { tail -30 gpurun_out/r3c_bench.log; exit 1; }
tail -1 gpurun_out/r3c_bench.log | cut -c1-400
