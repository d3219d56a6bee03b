# Round 3: Llama-3-70B TP=8 per-rank decode bench (collectives stubbed) + custom all-reduce microbench (same GPU, world 2/4/8)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u benchmarks/tp_rank_bench.py --model llama-3-70b --tp 8 --batch 8 --ctx 128 ${RANK_ARGS} > gpurun_out/r3_tp2_rank.log 2>&1 || { tail -30 gpurun_out/r3_tp2_rank.log; exit 1; }
grep '{' gpurun_out/r3_tp2_rank.log | tail -8
timeout -k 10 500 python -u benchmarks/allreduce_bench.py --worlds 2,4,8 --blocks 32,64,128 > gpurun_out/r3_tp2_ar.log 2>&1 || { tail -30 gpurun_out/r3_tp2_ar.log; exit 1; }
grep -c '{' gpurun_out/r3_tp2_ar.log
