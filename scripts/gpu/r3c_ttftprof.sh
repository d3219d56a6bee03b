# Round 3 (session 3): kernel stats of the Llama-3-8B TTFT probe (2048 and 4096-token prompts), summarised on the box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/ttftprof -o ttft -- python3 -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 2048 4096 --chunk 4096 > gpurun_out/r3c_ttftprof.log 2>&1 || { tail -30 gpurun_out/r3c_ttftprof.log; exit 1; }
grep '^{' gpurun_out/r3c_ttftprof.log
python3 benchmarks/prof_summary.py /tmp/ttftprof/ttft_results.db --top 30 > gpurun_out/r3c_ttftprof_kernels.txt
head -24 gpurun_out/r3c_ttftprof_kernels.txt | cut -c1-150
