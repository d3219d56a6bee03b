# Round 4: stream-K decode plans in context — Llama-3-70B TP8 per-rank step, Llama-3-8B decode timeline, plans off vs on
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u benchmarks/tp_rank_bench.py > gpurun_out/r4l_tp8.log 2>&1 || { tail -30 gpurun_out/r4l_tp8.log; exit 1; }
grep '^{' gpurun_out/r4l_tp8.log | cut -c1-1500
timeout -k 10 300 python -u benchmarks/timeline.py --model meta-llama/Meta-Llama-3-8B-Instruct --batch 8 --ctx 100 > gpurun_out/r4l_tl_llama8b.log 2>&1 || { tail -30 gpurun_out/r4l_tl_llama8b.log; exit 1; }
grep '"launches"' gpurun_out/r4l_tl_llama8b.log | cut -c1-1200
