# Round 5: fused QKV + attention + o_proj launch: tests, engine parity, same-box A/B (off / attention only / + o_proj)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "qkv_attention_fused" > gpurun_out/r5ac_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5ac_tests.log; exit 1; }
tail -1 gpurun_out/r5ac_tests.log
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5ac_engine.log 2>&1 || { echo E_FAIL; tail -60 gpurun_out/r5ac_engine.log; exit 1; }
tail -1 gpurun_out/r5ac_engine.log
run() {  # $1 = off / att / all, rest = script + args
  local f=$1; shift
  python -u -c "import sys, runpy; import vgate.ops as o; o.FUSE_QKV_ATTN = '$f' != 'off'; o.FUSE_OPROJ = '$f' == 'all'; sys.argv = sys.argv[1:]; runpy.run_path(sys.argv[0], run_name='__main__')" "$@"
}
for f in att all; do
timeout -k 10 300 bash -c "$(declare -f run); run $f benchmarks/timeline.py --batch 8 --ctx 100" > gpurun_out/r5ac_tl_$f.log 2>&1 || { tail -30 gpurun_out/r5ac_tl_$f.log; exit 1; }
grep -o '"launches": [0-9]*, "step_us": [0-9.]*, "sum_span_us": [0-9.]*, "sum_gap_us": [0-9.]*' gpurun_out/r5ac_tl_$f.log | head -1 | sed "s/^/$f /"
done
for f in att all; do
timeout -k 10 400 bash -c "$(declare -f run); run $f bench.py --gpus 1 --steps 20 --warmup 5" > gpurun_out/r5ac_bench_$f.log 2>&1 || { tail -30 gpurun_out/r5ac_bench_$f.log; exit 1; }
tail -1 gpurun_out/r5ac_bench_$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', {k: d.get(k) for k in ('value','p50_s','engine_avg_gpu_ms','timed_engine_idle_ms')})"
done
