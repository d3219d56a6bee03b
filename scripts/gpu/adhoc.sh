# ad-hoc GPU batch: TTFT at the final tree
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 512 2048 4096 > gpurun_out/fin_ttft.log 2>&1 || { tail -30 gpurun_out/fin_ttft.log; exit 1; }
grep '^{' gpurun_out/fin_ttft.log | tail -3
timeout -k 10 400 python -u benchmarks/ttft_probe.py --lens 512 2048 4096 > gpurun_out/fin_ttft_qwen.log 2>&1 || { tail -30 gpurun_out/fin_ttft_qwen.log; exit 1; }
grep '^{' gpurun_out/fin_ttft_qwen.log | tail -3
