# Round 4: tuned prefill plans at the long-prompt chunk sizes (1024 / 2048 rows): TTFT probe, Qwen2.5-1.5B + Llama-3-8B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u benchmarks/ttft_probe.py --lens 512 2048 4096 > gpurun_out/r4z_ttft_qwen.log 2>&1 || { tail -30 gpurun_out/r4z_ttft_qwen.log; exit 1; }
grep '^{' gpurun_out/r4z_ttft_qwen.log
timeout -k 10 500 python -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 512 2048 4096 > gpurun_out/r4z_ttft_llama.log 2>&1 || { tail -30 gpurun_out/r4z_ttft_llama.log; exit 1; }
grep '^{' gpurun_out/r4z_ttft_llama.log
