# Round 5 final: Llama-3-70B TP=8 rank step with the fused QKV + attention launch and the re-swept plans
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/tp_rank_bench.py > gpurun_out/r5am_tp8.log 2>&1 || { tail -30 gpurun_out/r5am_tp8.log; exit 1; }
timeout -k 10 300 python -u benchmarks/tp_rank_bench.py --fused-ar >> gpurun_out/r5am_tp8.log 2>&1 || { tail -30 gpurun_out/r5am_tp8.log; exit 1; }
grep '^{' gpurun_out/r5am_tp8.log | cut -c1-300
