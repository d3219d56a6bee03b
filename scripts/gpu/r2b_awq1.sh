set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention or awq" --timeout 120 --timeout-method thread > gpurun_out/r2b_awq_tests.log 2>&1 || { echo T_FAIL; tail -40 gpurun_out/r2b_awq_tests.log; exit 1; }
tail -2 gpurun_out/r2b_awq_tests.log
timeout -k 10 200 python -u benchmarks/attn_phases.py > gpurun_out/r2b_attn_phases3.log 2>&1 || { tail -30 gpurun_out/r2b_attn_phases3.log; exit 1; }
grep ctx gpurun_out/r2b_attn_phases3.log
timeout -k 10 400 python -u benchmarks/awq_sweep.py > gpurun_out/r2b_awq_sweep.log 2>&1 || { tail -30 gpurun_out/r2b_awq_sweep.log; exit 1; }
python - <<'PY'
import json
for line in open("gpurun_out/r2b_awq_sweep.log"):
    if not line.startswith("{"): continue
    d = json.loads(line)
    print(d["shape"], [(r["waves"], r["splitk"], r["ntb"], r["span_us"], r["wall_us"]) for r in d["rows"]])
PY
