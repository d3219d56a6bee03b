# A/B of two builds of the extension in one box session: $1 = label of the variant in ab/_C_base.so
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
SO=vgate/_C.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/new.so
run() {
  tag=$1
  timeout -k 10 200 python -u benchmarks/attn_phases.py > gpurun_out/r2b_ab_phases_$tag.log 2>&1 || { tail -30 gpurun_out/r2b_ab_phases_$tag.log; exit 1; }
  echo "== $tag"; grep ctx gpurun_out/r2b_ab_phases_$tag.log | cut -c1-200
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r2b_ab_bench_$tag.log 2>&1 || { tail -30 gpurun_out/r2b_ab_bench_$tag.log; exit 1; }
  tail -1 gpurun_out/r2b_ab_bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','p50_s','p99_s','engine_avg_gpu_ms')})"
}
run new1
cp ab/_C_base.so $SO
run base1
cp /tmp/new.so $SO
run new2
cp ab/_C_base.so $SO
run base2
cp /tmp/new.so $SO
