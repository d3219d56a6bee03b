set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "gemm or engine" --timeout 120 --timeout-method thread > gpurun_out/r2b_u6_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r2b_u6_tests.log; exit 1; }
tail -1 gpurun_out/r2b_u6_tests.log
for u in 0 8 0 8; do
  timeout -k 10 300 env VGATE_DEC_U=$u python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r2b_u6_tl_$u.log 2>&1 || { tail -30 gpurun_out/r2b_u6_tl_$u.log; exit 1; }
  echo "U=$u"; grep -v '^{"kernel"' gpurun_out/r2b_u6_tl_$u.log | grep '^{' | python -c "
import json,sys
t=json.loads(sys.stdin.read().splitlines()[-1]); print(t['step_us'], {k: (v['avg_span_us'], v['avg_gap_after_us']) for k,v in t['per_kernel'].items() if k.startswith('gemm')})"
done
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','p50_s','p99_s')})"; }
for t in u6a:0 u8a:8 u6b:0 u8b:8; do
  tag=${t%%:*}; u=${t##*:}
  timeout -k 10 300 env VGATE_DEC_U=$u python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2b_u6_$tag.log 2>&1 || { tail -30 gpurun_out/r2b_u6_$tag.log; exit 1; }
  echo -n "$tag "; summ gpurun_out/r2b_u6_$tag.log
done
