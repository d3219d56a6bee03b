# Round 3 (session 2): medium-M kernels (split + wide) — correctness, cold-cache shape sweep, in-engine mixed steps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "mid_gemm or mid_wide or prefill_lds_gemm or tune_prefill" > gpurun_out/r3b_mid2_tests.log 2>&1 || { tail -40 gpurun_out/r3b_mid2_tests.log; exit 1; }
tail -2 gpurun_out/r3b_mid2_tests.log
timeout -k 10 400 python -u benchmarks/medium_m_bench.py --iters 6 > gpurun_out/r3b_mid2_mm.log 2>&1 || { tail -30 gpurun_out/r3b_mid2_mm.log; exit 1; }
python3 - gpurun_out/r3b_mid2_mm.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        a = d["all"]
        mids = {k: v for k, v in a.items() if k.startswith("-1")}
        bm = min(mids, key=mids.get) if mids else None
        print(d["shape"], d["M"], "default", d["default_us"], "best", d["best"], d["best_us"], "best_mid", bm, mids.get(bm), "wide", a.get("-18/0"))
PY
for m in default tuned; do
timeout -k 10 300 python -u benchmarks/mixed_step.py --medium $m --prompts 16,32,48 > gpurun_out/r3b_mid2_mixed_$m.log 2>&1 || { tail -30 gpurun_out/r3b_mid2_mixed_$m.log; exit 1; }
grep '^{' gpurun_out/r3b_mid2_mixed_$m.log | cut -c1-700
done
