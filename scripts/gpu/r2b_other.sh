set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --model meta-llama/Meta-Llama-3-8B-Instruct > gpurun_out/r2b_other_llama8b.log 2>&1 || { tail -30 gpurun_out/r2b_other_llama8b.log; exit 1; }
tail -1 gpurun_out/r2b_other_llama8b.log | cut -c1-600
timeout -k 10 300 python -u benchmarks/ttft_probe.py --lens 512 2048 4096 --chunk 4096 > gpurun_out/r2b_other_ttft_qwen.log 2>&1 || { tail -30 gpurun_out/r2b_other_ttft_qwen.log; exit 1; }
grep ttft_ms gpurun_out/r2b_other_ttft_qwen.log | cut -c1-250
