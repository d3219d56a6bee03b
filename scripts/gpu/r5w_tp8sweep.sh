# Round 5: Llama-3-70B TP=8 rank in-context sweep with the register-stationary and stream-K candidates
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u benchmarks/tp_rank_bench.py --sweep --iters 30 > gpurun_out/r5w_tp8sweep.log 2>&1 || { tail -30 gpurun_out/r5w_tp8sweep.log; exit 1; }
grep '^{' gpurun_out/r5w_tp8sweep.log | cut -c1-300
