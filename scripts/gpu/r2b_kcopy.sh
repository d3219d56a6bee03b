set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_tp_gpu.py -x -q -k "kernel_copy or engine or tp" --timeout 120 --timeout-method thread > gpurun_out/r2b_kc_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r2b_kc_tests.log; exit 1; }
tail -1 gpurun_out/r2b_kc_tests.log
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','engine_avg_step_ms')})"; }
b() {
  tag=$1; shift
  timeout -k 10 300 env "$@" python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2b_kc_$tag.log 2>&1 || { tail -30 gpurun_out/r2b_kc_$tag.log; exit 1; }
  echo -n "$tag "; summ gpurun_out/r2b_kc_$tag.log
}
b kc1 VGATE_KERNEL_COPY=1
b memcpy1 VGATE_KERNEL_COPY=0
b kc2 VGATE_KERNEL_COPY=1
b memcpy2 VGATE_KERNEL_COPY=0
rm -rf gpurun_out/prof_k
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_k -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/r2b_kc_prof.log 2>&1 || { tail -30 gpurun_out/r2b_kc_prof.log; exit 1; }
DB=$(find gpurun_out/prof_k -name "*results.db" | head -1)
python benchmarks/trace_gaps.py $DB --first 4 > gpurun_out/r2b_kc_gaps.log 2>&1 || { cat gpurun_out/r2b_kc_gaps.log; exit 1; }
cat gpurun_out/r2b_kc_gaps.log | cut -c1-300
mv $DB gpurun_out/r2b_kc_trace.db; rm -rf gpurun_out/prof_k
