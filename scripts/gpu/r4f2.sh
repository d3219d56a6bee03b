# Round 4 HEAD evidence (2/2): AWQ + security bench, Llama-3-8B HTTP bench / bench_compare, TTFT (Qwen, Llama-3-8B), flash prefill bench,
# single-request TTFT with the idle admission window on / off
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r4f2_awq.log 2>&1 || { tail -30 gpurun_out/r4f2_awq.log; exit 1; }
tail -1 gpurun_out/r4f2_awq.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('awq', {k: d.get(k) for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','dtype')})"
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 --model meta-llama/Meta-Llama-3-8B-Instruct > gpurun_out/r4f2_llama8b.log 2>&1 || { tail -30 gpurun_out/r4f2_llama8b.log; exit 1; }
tail -1 gpurun_out/r4f2_llama8b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('llama8b', {k: d.get(k) for k in ('value','p50_s','p99_s','engine_avg_gpu_ms')})"
VGATE_MODEL__MODEL_ID=meta-llama/Meta-Llama-3-8B-Instruct timeout -k 10 500 python -u benchmarks/bench_compare.py --backends native --prompts 8 --rounds 3 --output json > gpurun_out/r4f2_compare_llama8b.log 2>&1 || { tail -30 gpurun_out/r4f2_compare_llama8b.log; exit 1; }
tail -3 gpurun_out/r4f2_compare_llama8b.log | cut -c1-400
timeout -k 10 400 python -u benchmarks/ttft_probe.py --model Qwen/Qwen2.5-1.5B-Instruct --lens 512 2048 4096 --chunk 4096 > gpurun_out/r4f2_ttft_qwen.log 2>&1 || { tail -30 gpurun_out/r4f2_ttft_qwen.log; exit 1; }
grep '^{' gpurun_out/r4f2_ttft_qwen.log | cut -c1-220
timeout -k 10 500 python -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 512 2048 4096 --chunk 4096 > gpurun_out/r4f2_ttft_llama.log 2>&1 || { tail -30 gpurun_out/r4f2_ttft_llama.log; exit 1; }
grep '^{' gpurun_out/r4f2_ttft_llama.log | cut -c1-220
timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py --lens 1024,2048,4096,8192 > gpurun_out/r4f2_flash.log 2>&1 || { tail -30 gpurun_out/r4f2_flash.log; exit 1; }
grep '^{' gpurun_out/r4f2_flash.log | cut -c1-160
for w in 3.0 0; do
VGATE_IDLE_BATCH_WINDOW_MS=$w timeout -k 10 300 python -u benchmarks/ttft_probe.py --model Qwen/Qwen2.5-1.5B-Instruct --lens 64 512 --chunk 2048 > gpurun_out/r4f2_ttft_window_$w.log 2>&1 || { tail -30 gpurun_out/r4f2_ttft_window_$w.log; exit 1; }
echo "idle window $w ms:"; grep '^{' gpurun_out/r4f2_ttft_window_$w.log | cut -c1-220
done
