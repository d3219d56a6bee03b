# Round 4: stream-K decode GEMM — numerics, then decode timelines A/B (tile-per-block vs stream-K)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_streamk_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4i_tests.log 2>&1 || { echo TEST_FAIL; tail -60 gpurun_out/r4i_tests.log; exit 1; }
tail -3 gpurun_out/r4i_tests.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r4i_timeline_base.log 2>&1 || { tail -30 gpurun_out/r4i_timeline_base.log; exit 1; }
grep '"launches"' gpurun_out/r4i_timeline_base.log | cut -c1-200
VGATE_STREAMK=1 timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r4i_timeline_sk.log 2>&1 || { tail -30 gpurun_out/r4i_timeline_sk.log; exit 1; }
grep '"launches"' gpurun_out/r4i_timeline_sk.log | cut -c1-200
python - <<'PY'
import json
for f in ("gpurun_out/r4i_timeline_base.log", "gpurun_out/r4i_timeline_sk.log"):
    for l in open(f):
        if l.startswith('{"kv_blocks'):
            d = json.loads(l)
            print(f, d["step_us"], d["launches"])
            for k, v in d["per_kernel"].items():
                print("  ", k, v["n"], v["avg_span_us"], v["avg_gap_after_us"], v["dur_med"], v["dur_max"])
PY
