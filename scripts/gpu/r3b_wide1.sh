# Round 3 (session 2): wide medium kernel at decode M (one block per CU, x once per CU in LDS) — tests, cold shapes, in-engine gate_up sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "mid_wide or mid_gemm_plans" > gpurun_out/r3b_wide1_tests.log 2>&1 || { tail -40 gpurun_out/r3b_wide1_tests.log; exit 1; }
tail -1 gpurun_out/r3b_wide1_tests.log
timeout -k 10 400 python -u benchmarks/medium_m_bench.py --iters 6 --ms 8,16,64 > gpurun_out/r3b_wide1_mm.log 2>&1 || { tail -30 gpurun_out/r3b_wide1_mm.log; exit 1; }
python3 - gpurun_out/r3b_wide1_mm.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        a = d["all"]
        print(d["shape"], d["M"], "default", d["default_us"], "wide", a.get("-18/0"), "best", d["best"], d["best_us"])
PY
timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --kinds gate_up > gpurun_out/r3b_wide1_sweep.log 2>&1 || { tail -30 gpurun_out/r3b_wide1_sweep.log; exit 1; }
grep '^{' gpurun_out/r3b_wide1_sweep.log | head -5
