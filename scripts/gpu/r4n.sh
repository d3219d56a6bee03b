# Round 4: prefill-step timeline (8 prompts x 50 tokens, one multi-prompt step) at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/timeline.py --prefill --batch 8 --ctx 50 > gpurun_out/r4n_tl_prefill.log 2>&1 || { tail -30 gpurun_out/r4n_tl_prefill.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r4n_tl_prefill.log"):
    if l.startswith('{"kv_blocks'):
        d = json.loads(l)
        print(d["step_us"], d["launches"], d["sum_gap_us"])
        for k, v in d["per_kernel"].items():
            print("  ", k, v["n"], v["avg_span_us"], v["avg_gap_after_us"], v["dur_med"], v["dur_max"])
PY
