# Round 3 (session 2): AWQ mixed steps (tuned medium plans on the dequant scratch) + AWQ decode timeline with the new plans
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/mixed_step.py --quantization awq --prompts 16,32,48 > gpurun_out/r3b_awqmix.log 2>&1 || { tail -30 gpurun_out/r3b_awqmix.log; exit 1; }
grep '^{"case' gpurun_out/r3b_awqmix.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 7 --ctx 100 --mixed 48 --quantization awq > gpurun_out/r3b_awqmix_tl.log 2>&1 || { tail -30 gpurun_out/r3b_awqmix_tl.log; exit 1; }
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 --quantization awq > gpurun_out/r3b_awqdec_tl.log 2>&1 || { tail -30 gpurun_out/r3b_awqdec_tl.log; exit 1; }
for f in gpurun_out/r3b_awqmix_tl.log gpurun_out/r3b_awqdec_tl.log; do
python - $f <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith('{"kv_blocks"'):
        d = json.loads(ln)
        print(sys.argv[1], "step_us", d["step_us"], "gaps", d["sum_gap_us"])
        for k, v in d["per_kernel"].items():
            if v["n"] >= 28: print("  ", k, "span", v["avg_span_us"], "gap", v["avg_gap_after_us"], "dur p10/med/max", v["dur_p10"], v["dur_med"], v["dur_max"])
PY
done
