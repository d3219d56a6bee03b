# Round 4: Llama-3-8B 2000-token prefill step timeline (where TTFT@2048 goes) + TTFT probe
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u benchmarks/timeline.py --model meta-llama/Meta-Llama-3-8B-Instruct --prefill --batch 1 --ctx 2000 --max-seqs 8 > gpurun_out/r4x_llama_prefill_tl.log 2>&1 || { tail -30 gpurun_out/r4x_llama_prefill_tl.log; exit 1; }
head -c 6000 gpurun_out/r4x_llama_prefill_tl.log
timeout -k 10 500 python -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 2048 > gpurun_out/r4x_llama_ttft.log 2>&1 || { tail -30 gpurun_out/r4x_llama_ttft.log; exit 1; }
grep '^{' gpurun_out/r4x_llama_ttft.log
