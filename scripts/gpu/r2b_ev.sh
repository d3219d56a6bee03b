set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_tp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2b_ev_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r2b_ev_tests.log; exit 1; }
tail -1 gpurun_out/r2b_ev_tests.log
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','engine_avg_step_ms')})"; }
b() {
  tag=$1; shift
  timeout -k 10 300 env "$@" python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2b_ev_$tag.log 2>&1 || { tail -30 gpurun_out/r2b_ev_$tag.log; exit 1; }
  echo -n "$tag "; summ gpurun_out/r2b_ev_$tag.log
}
b timing1 VGATE_STEP_TIMING=1
b notiming1 VGATE_STEP_TIMING=0
b timing2 VGATE_STEP_TIMING=1
b notiming2 VGATE_STEP_TIMING=0
rm -rf gpurun_out/prof_e
timeout -k 10 400 env VGATE_STEP_TIMING=0 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_e -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/r2b_ev_prof.log 2>&1 || { tail -30 gpurun_out/r2b_ev_prof.log; exit 1; }
DB=$(find gpurun_out/prof_e -name "*results.db" | head -1)
mv $DB gpurun_out/r2b_ev_trace.db; rm -rf gpurun_out/prof_e
