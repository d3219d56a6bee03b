# Round 4: same-box A/B of the TP=1 decode step before (26077c9, ab_old/) and after the fused TP epilogue (HEAD)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  (cd ab_old && timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only > ../gpurun_out/r4ab_old_$i.log 2>&1) || { tail -20 gpurun_out/r4ab_old_$i.log; exit 1; }
  echo "old $i"; grep '^{' gpurun_out/r4ab_old_$i.log
  timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only > gpurun_out/r4ab_new_$i.log 2>&1 || { tail -20 gpurun_out/r4ab_new_$i.log; exit 1; }
  echo "new $i"; grep '^{' gpurun_out/r4ab_new_$i.log
done
