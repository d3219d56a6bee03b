# Round 3 (session 2): in-graph launch timeline of the P=48 mixed step (block durations per kernel), tuned vs wide gate_up
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" "--wide-gate-up"; do
timeout -k 10 300 python -u benchmarks/timeline.py --batch 7 --ctx 100 --mixed 48 $v > gpurun_out/r3b_mid4$v.log 2>&1 || { tail -30 gpurun_out/r3b_mid4$v.log; exit 1; }
python - gpurun_out/r3b_mid4$v.log <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith('{"kv_blocks"'):
        d = json.loads(ln)
        print("step_us", d["step_us"], "gaps", d["sum_gap_us"])
        for k, v in d["per_kernel"].items():
            if v["n"] >= 28: print("  ", k, "span", v["avg_span_us"], "gap", v["avg_gap_after_us"], "dur p10/med/max", v["dur_p10"], v["dur_med"], v["dur_max"], "start_max", v["start_max"])
PY
done
