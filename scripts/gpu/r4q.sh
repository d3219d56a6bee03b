# Round 4: prefill tile sweep at the 448-row bucket (Qwen2.5-1.5B, all tile / split candidates, hot back-to-back timing as the tuner)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u benchmarks/prefill_tile_sweep.py --ms 448 --model qwen --tiles 0,64,128,256,768,1024,1280,1281,640,641 --sks 0,2,3,4,6 > gpurun_out/r4q_sweep448.log 2>&1 || { tail -30 gpurun_out/r4q_sweep448.log; exit 1; }
cut -c1-1500 gpurun_out/r4q_sweep448.log | grep '^{'
for rl in 0 2; do
VGATE_SAMPLE_ROUND_LAUNCHES=$rl timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r4q_tl_rl$rl.log 2>&1 || { tail -30 gpurun_out/r4q_tl_rl$rl.log; exit 1; }
python - <<PY
import json
for l in open("gpurun_out/r4q_tl_rl$rl.log"):
    if l.startswith('{"kv_blocks'):
        d = json.loads(l)
        print("round launches $rl step", d["step_us"], d["launches"])
        for k, v in d["per_kernel"].items():
            if "sample" in k: print("  ", k, v["n"], v["avg_span_us"], v["dur_med"], v["dur_max"])
PY
done
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "awq" -x -q --timeout 120 --timeout-method thread > gpurun_out/r4q_awq_tests.log 2>&1 || { echo AWQ_TEST_FAIL; tail -40 gpurun_out/r4q_awq_tests.log; exit 1; }
tail -1 gpurun_out/r4q_awq_tests.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 --quantization awq > gpurun_out/r4q_tl_awq.log 2>&1 || { tail -30 gpurun_out/r4q_tl_awq.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r4q_tl_awq.log"):
    if l.startswith('{"kv_blocks'):
        d = json.loads(l)
        print("awq step", d["step_us"])
        for k, v in list(d["per_kernel"].items())[:5]:
            print("  ", k, v["n"], v["avg_span_us"], v["dur_med"], v["dur_max"])
PY
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq > gpurun_out/r4q_awq_bench.log 2>&1 || { tail -30 gpurun_out/r4q_awq_bench.log; exit 1; }
tail -1 gpurun_out/r4q_awq_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('awq (no security)', {k: d.get(k) for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','dtype')})"
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4q_bf16_bench.log 2>&1 || { tail -30 gpurun_out/r4q_bf16_bench.log; exit 1; }
tail -1 gpurun_out/r4q_bf16_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bf16 same box', {k: d.get(k) for k in ('value','p50_s','p99_s','engine_avg_gpu_ms')})"
