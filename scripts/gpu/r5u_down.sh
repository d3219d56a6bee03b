# Round 5: bf16 down_proj decompositions (tile kernel waves / slices, stream-K, register-stationary)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
DKX_SHAPES=down timeout -k 10 300 python -u benchmarks/dense_kx_sweep.py > gpurun_out/r5u_down.log 2>&1 || { tail -30 gpurun_out/r5u_down.log; exit 1; }
echo ok
timeout -k 10 300 python -u benchmarks/timeline.py --prefill --batch 8 --ctx 50 > gpurun_out/r5u_prefill_timeline.log 2>&1 || { tail -30 gpurun_out/r5u_prefill_timeline.log; exit 1; }
grep -h '"step_us"' gpurun_out/r5u_prefill_timeline.log | cut -c1-120
