# Round 4: stream-K (early lead publish) vs the tile-per-block kernels, per projection (cold weights, in-graph)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_streamk_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4k_tests.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/r4k_tests.log; exit 1; }
tail -1 gpurun_out/r4k_tests.log
for m in qwen llama70b_tp8 llama8b; do
  timeout -k 10 300 python -u benchmarks/sk_probe.py --model $m > gpurun_out/r4k_probe_$m.log 2>&1 || { tail -30 gpurun_out/r4k_probe_$m.log; exit 1; }
  grep '^{' gpurun_out/r4k_probe_$m.log
done
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k sample -x -q --timeout 120 --timeout-method thread > gpurun_out/r4k_sample_tests.log 2>&1 || { echo SAMPLE_TEST_FAIL; tail -40 gpurun_out/r4k_sample_tests.log; exit 1; }
tail -1 gpurun_out/r4k_sample_tests.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r4k_timeline.log 2>&1 || { tail -30 gpurun_out/r4k_timeline.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r4k_timeline.log"):
    if l.startswith('{"kv_blocks'):
        d = json.loads(l)
        print(d["step_us"], d["launches"])
        for k, v in d["per_kernel"].items():
            if "sample" in k: print("  ", k, v["n"], v["avg_span_us"], v["avg_gap_after_us"], v["dur_med"], v["dur_max"])
PY
