# Round 3 (session 3): kernel stats of the Llama-3-8B TTFT probe (2048 and 4096-token prompts)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/ttftprof -o ttft -- python3 -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 2048 4096 --chunk 4096 > gpurun_out/r3c_ttftprof.log 2>&1 || { tail -30 gpurun_out/r3c_ttftprof.log; exit 1; }
grep '^{' gpurun_out/r3c_ttftprof.log
f=$(find /tmp/ttftprof -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/r3c_ttftprof_kernel_stats.csv
head -25 "$f" | cut -c1-220
VGATE_FLASH_CT=2 timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py --lens 1024,2048,4096,8192 > gpurun_out/r3c_flash_ct2split.log 2>&1 || { tail -30 gpurun_out/r3c_flash_ct2split.log; exit 1; }
echo "CT=2 + split"; grep '^{' gpurun_out/r3c_flash_ct2split.log | grep qwen | cut -c1-200
