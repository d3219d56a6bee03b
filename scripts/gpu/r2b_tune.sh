set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2b_tune_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r2b_tune_tests.log; exit 1; }
tail -1 gpurun_out/r2b_tune_tests.log
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','max_gpu_step_ms')})"; }
b() {
  tag=$1; shift
  timeout -k 10 300 env "$@" python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2b_tune_$tag.log 2>&1 || { tail -30 gpurun_out/r2b_tune_$tag.log; exit 1; }
  echo -n "$tag "; summ gpurun_out/r2b_tune_$tag.log
  grep -h "prefill GEMM plans" gpurun_out/r2b_tune_$tag.log | cut -c1-600 | head -1
}
b tune1 VGATE_PREFILL_AUTOTUNE=1
b heur1 VGATE_PREFILL_AUTOTUNE=0
b tune2 VGATE_PREFILL_AUTOTUNE=1
b heur2 VGATE_PREFILL_AUTOTUNE=0
