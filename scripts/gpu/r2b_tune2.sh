set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "awq" --timeout 120 --timeout-method thread > gpurun_out/r2b_tune2_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r2b_tune2_tests.log; exit 1; }
tail -1 gpurun_out/r2b_tune2_tests.log
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','max_gpu_step_ms')})"; }
b() {
  tag=$1; shift
  timeout -k 10 300 env "$@" python -u bench.py --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r2b_tune2_$tag.log 2>&1 || { tail -30 gpurun_out/r2b_tune2_$tag.log; exit 1; }
  echo -n "$tag "; summ gpurun_out/r2b_tune2_$tag.log
}
b awq_tune1 VGATE_PREFILL_AUTOTUNE=1
b awq_heur1 VGATE_PREFILL_AUTOTUNE=0
b awq_tune2 VGATE_PREFILL_AUTOTUNE=1
for t in 1 0; do
  timeout -k 10 400 env VGATE_PREFILL_AUTOTUNE=$t python -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 2048 4096 --chunk 4096 > gpurun_out/r2b_tune2_ttft$t.log 2>&1 || { tail -30 gpurun_out/r2b_tune2_ttft$t.log; exit 1; }
  echo "autotune=$t"; grep ttft_ms gpurun_out/r2b_tune2_ttft$t.log | cut -c1-300
done
