# Round 3: Llama-3-70B TP=8 per-rank decode decomposition sweep (collectives stubbed)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u benchmarks/tp_rank_bench.py --model llama-3-70b --tp 8 --batch 8 --ctx 128 --sweep --iters 30 > gpurun_out/r3_tp3_sweep.log 2>&1 || { tail -30 gpurun_out/r3_tp3_sweep.log; exit 1; }
grep '"best"' gpurun_out/r3_tp3_sweep.log
