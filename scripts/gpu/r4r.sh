# Round 4: decode split-K combined through granules (last slice collects) — numerics, decode timelines bf16 / AWQ, driver bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_streamk_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4r_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/r4r_tests.log; exit 1; }
tail -1 gpurun_out/r4r_tests.log
for q in none awq; do
  if [ $q = none ]; then QA=""; else QA="--quantization awq"; fi
  timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 $QA > gpurun_out/r4r_tl_$q.log 2>&1 || { tail -30 gpurun_out/r4r_tl_$q.log; exit 1; }
  python - <<PY
import json
for l in open("gpurun_out/r4r_tl_$q.log"):
    if l.startswith('{"kv_blocks'):
        d = json.loads(l)
        print("$q step", d["step_us"], d["launches"])
        for k, v in list(d["per_kernel"].items())[:6]:
            print("  ", k, v["n"], v["avg_span_us"], v["dur_med"], v["dur_max"])
PY
done
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4r_bench.log 2>&1 || { tail -30 gpurun_out/r4r_bench.log; exit 1; }
tail -1 gpurun_out/r4r_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','p50_s','p99_s','engine_avg_gpu_ms')})"
