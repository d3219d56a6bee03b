# Round 4: smaller tuner margin for >= 1024-row chunks: TTFT Llama-3-8B / Qwen2.5-1.5B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 512 2048 4096 --chunk 4096 > gpurun_out/r4aj_ttft_llama.log 2>&1 || { tail -30 gpurun_out/r4aj_ttft_llama.log; exit 1; }
grep '^{' gpurun_out/r4aj_ttft_llama.log | cut -c1-220
timeout -k 10 400 python -u benchmarks/ttft_probe.py --lens 512 2048 4096 --chunk 4096 > gpurun_out/r4aj_ttft_qwen.log 2>&1 || { tail -30 gpurun_out/r4aj_ttft_qwen.log; exit 1; }
grep '^{' gpurun_out/r4aj_ttft_qwen.log | cut -c1-220
