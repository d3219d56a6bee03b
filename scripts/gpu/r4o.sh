# Round 4: epilogue-operand prefetch in the int4 stream kernel and in stream-K — numerics, AWQ decode timeline, stream-K probe (Qwen, 8B)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_streamk_gpu.py tests/test_kernels_gpu.py -k "streamk or awq" -x -q --timeout 120 --timeout-method thread > gpurun_out/r4o_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/r4o_tests.log; exit 1; }
tail -1 gpurun_out/r4o_tests.log
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4o_engine.log 2>&1 || { echo ENGINE_FAIL; tail -60 gpurun_out/r4o_engine.log; exit 1; }
tail -1 gpurun_out/r4o_engine.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 --quantization awq > gpurun_out/r4o_tl_awq.log 2>&1 || { tail -30 gpurun_out/r4o_tl_awq.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r4o_tl_awq.log"):
    if l.startswith('{"kv_blocks'):
        d = json.loads(l)
        print("awq step", d["step_us"], d["launches"])
        for k, v in d["per_kernel"].items():
            print("  ", k, v["n"], v["avg_span_us"], v["avg_gap_after_us"], v["dur_med"], v["dur_max"])
PY
for m in qwen llama8b; do
  timeout -k 10 300 python -u benchmarks/sk_probe.py --model $m > gpurun_out/r4o_probe_$m.log 2>&1 || { tail -30 gpurun_out/r4o_probe_$m.log; exit 1; }
  grep '^{' gpurun_out/r4o_probe_$m.log
done
timeout -k 10 300 python -u benchmarks/timeline.py --prefill --batch 8 --ctx 50 > gpurun_out/r4o_tl_prefill.log 2>&1 || { tail -30 gpurun_out/r4o_tl_prefill.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r4o_tl_prefill.log"):
    if l.startswith('{"kv_blocks'):
        d = json.loads(l)
        print("prefill step", d["step_us"], d["launches"], d["sum_gap_us"])
        for k, v in list(d["per_kernel"].items())[:8]:
            print("  ", k, v["n"], v["avg_span_us"], v["avg_gap_after_us"])
PY
for dv in 1 4; do
VGATE_SAMPLE_RESUME_DIV=$dv timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r4o_tl_div$dv.log 2>&1 || { tail -30 gpurun_out/r4o_tl_div$dv.log; exit 1; }
python - <<PY
import json
for l in open("gpurun_out/r4o_tl_div$dv.log"):
    if l.startswith('{"kv_blocks'):
        d = json.loads(l)
        print("div $dv step", d["step_us"])
        for k, v in d["per_kernel"].items():
            if "sample" in k: print("  ", k, v["avg_span_us"], v["dur_med"], v["dur_max"])
PY
done
