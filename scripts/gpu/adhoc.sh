# ad-hoc GPU batch: TTFT with every timed token prefilled, and the rounds 3-6 prompts (shared prefix) for comparison
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for m in meta-llama/Meta-Llama-3-8B-Instruct Qwen/Qwen2.5-1.5B-Instruct; do
for f in "" "--shared-prefix"; do
timeout -k 10 400 python -u benchmarks/ttft_probe.py --model $m --lens 512 2048 4096 $f > gpurun_out/fix2_ttft.log 2>&1 || { tail -30 gpurun_out/fix2_ttft.log; exit 1; }
echo "# $m ${f:-unique prompts}"; grep '^{' gpurun_out/fix2_ttft.log | tail -3
done
done
