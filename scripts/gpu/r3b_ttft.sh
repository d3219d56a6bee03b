# Round 3 (session 2): TTFT at HEAD (engine-level), Qwen2.5-1.5B and Llama-3-8B, 512 / 2048 / 4096-token prompts; flash prefill bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u benchmarks/ttft_probe.py --model Qwen/Qwen2.5-1.5B-Instruct --lens 512 2048 4096 --chunk 4096 > gpurun_out/r3b_ttft_qwen.log 2>&1 || { tail -30 gpurun_out/r3b_ttft_qwen.log; exit 1; }
grep '^{' gpurun_out/r3b_ttft_qwen.log
timeout -k 10 500 python -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 512 2048 4096 --chunk 4096 > gpurun_out/r3b_ttft_llama.log 2>&1 || { tail -30 gpurun_out/r3b_ttft_llama.log; exit 1; }
grep '^{' gpurun_out/r3b_ttft_llama.log
timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py > gpurun_out/r3b_attn_prefill.log 2>&1 || { tail -30 gpurun_out/r3b_attn_prefill.log; exit 1; }
grep '^{' gpurun_out/r3b_attn_prefill.log | cut -c1-200
