# Round 5: same-box A/B of the fused QKV + attention launch (ops.FUSE_QKV_ATTN) — decode timeline and driver bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # $1 = on/off, rest = script + args
  local f=$1; shift
  python -u -c "import sys, runpy; import vgate.ops as o; o.FUSE_QKV_ATTN = ('$f' == 'on'); sys.argv = sys.argv[1:]; runpy.run_path(sys.argv[0], run_name='__main__')" "$@"
}
for f in off on; do
timeout -k 10 300 bash -c "$(declare -f run); run $f benchmarks/timeline.py --batch 8 --ctx 100" > gpurun_out/r5ab_tl_$f.log 2>&1 || { tail -30 gpurun_out/r5ab_tl_$f.log; exit 1; }
grep -o '"step_us": [0-9.]*, "sum_span_us": [0-9.]*, "sum_gap_us": [0-9.]*' gpurun_out/r5ab_tl_$f.log | head -1 | sed "s/^/$f /"
done
for i in 1 2; do for f in off on; do
timeout -k 10 400 bash -c "$(declare -f run); run $f bench.py --gpus 1 --steps 20 --warmup 5" > gpurun_out/r5ab_bench_${f}_$i.log 2>&1 || { tail -30 gpurun_out/r5ab_bench_${f}_$i.log; exit 1; }
tail -1 gpurun_out/r5ab_bench_${f}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', {k: d.get(k) for k in ('value','p50_s','engine_avg_gpu_ms','timed_engine_idle_ms')})"
done; done
