set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "gemm or engine" --timeout 120 --timeout-method thread > gpurun_out/r2b_tail_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r2b_tail_tests.log; exit 1; }
tail -1 gpurun_out/r2b_tail_tests.log
for t in 1 0 1 0; do
  timeout -k 10 300 env VGATE_TAIL_SPLIT=$t python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r2b_tail_tl_$t.log 2>&1 || { tail -30 gpurun_out/r2b_tail_tl_$t.log; exit 1; }
  echo "TAIL=$t"; grep -v '^{"kernel"' gpurun_out/r2b_tail_tl_$t.log | grep '^{' | python -c "
import json,sys
t=json.loads(sys.stdin.read().splitlines()[-1]); print(t['step_us'], {k: (v['avg_span_us'], v['avg_gap_after_us']) for k,v in t['per_kernel'].items() if k.startswith('gemm')})"
done
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','p50_s','p99_s')})"; }
for t in a:1 b:0 c:1 d:0; do
  tag=${t%%:*}; v=${t##*:}
  timeout -k 10 300 env VGATE_TAIL_SPLIT=$v python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2b_tail_$tag.log 2>&1 || { tail -30 gpurun_out/r2b_tail_$tag.log; exit 1; }
  echo -n "tail=$v "; summ gpurun_out/r2b_tail_$tag.log
done
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "awq" --timeout 120 --timeout-method thread > gpurun_out/r2b_tail_awq_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r2b_tail_awq_tests.log; exit 1; }
tail -1 gpurun_out/r2b_tail_awq_tests.log
for t in a:1 b:0; do
  tag=${t%%:*}; v=${t##*:}
  timeout -k 10 300 env VGATE_TAIL_SPLIT=$v python -u bench.py --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r2b_tail_awq_$tag.log 2>&1 || { tail -30 gpurun_out/r2b_tail_awq_$tag.log; exit 1; }
  echo -n "awq tail=$v "; summ gpurun_out/r2b_tail_awq_$tag.log
done
