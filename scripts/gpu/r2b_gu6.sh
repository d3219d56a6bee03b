set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for u in 6 0 6 0; do
  timeout -k 10 300 env VGATE_DEC_U=$u python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r2b_gu6_tl_$u.log 2>&1 || { tail -30 gpurun_out/r2b_gu6_tl_$u.log; exit 1; }
  echo "U=$u"; grep -v '^{"kernel"' gpurun_out/r2b_gu6_tl_$u.log | grep '^{' | python -c "
import json,sys
t=json.loads(sys.stdin.read().splitlines()[-1]); print(t['step_us'], {k: (v['avg_span_us'], v['avg_gap_after_us']) for k,v in t['per_kernel'].items() if k.startswith('gemm')})"
done
