# Round 3 (session 2): HEAD sanity — GPU tier, smoke, driver bench, AWQ bench, decode timelines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r3b_base_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r3b_base_tests.log; exit 1; }
tail -1 gpurun_out/r3b_base_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3b_base_smoke.log 2>&1 || { tail -30 gpurun_out/r3b_base_smoke.log; exit 1; }
tail -1 gpurun_out/r3b_base_smoke.log | cut -c1-160
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3b_base_bench.log 2>&1 || { tail -30 gpurun_out/r3b_base_bench.log; exit 1; }
tail -1 gpurun_out/r3b_base_bench.log | cut -c1-400
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r3b_base_awq.log 2>&1 || { tail -30 gpurun_out/r3b_base_awq.log; exit 1; }
tail -1 gpurun_out/r3b_base_awq.log | cut -c1-400
for q in none awq; do
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 --quantization $q > gpurun_out/r3b_base_timeline_$q.log 2>&1 || { tail -30 gpurun_out/r3b_base_timeline_$q.log; exit 1; }
python - gpurun_out/r3b_base_timeline_$q.log <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith('{"batch"'):
        d = json.loads(ln)
        print("step_us", d["step_us"], {k: (v["avg_span_us"], v["avg_gap_after_us"], v["dur_med"]) for k, v in d["per_kernel"].items()})
PY
done
