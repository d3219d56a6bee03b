# Round 3: price the decode GEMMs' activation loads in-engine (VGATE_GEMM_PROBE=1 skips them),
# for the one-tile-per-block kernels and the balanced gate_up kernel; timelines per mode
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "0 0" "1 0" "0 1" "1 1"; do
  set -- $cfg
  VGATE_GEMM_PROBE=$1 VGATE_DEC_BAL=$2 timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r3_probe1_p$1_b$2.log 2>&1 || { tail -30 gpurun_out/r3_probe1_p$1_b$2.log; exit 1; }
  python - gpurun_out/r3_probe1_p$1_b$2.log $1 $2 <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith('{"batch"'):
        d = json.loads(ln)
        pk = {k: (v["avg_span_us"], v["avg_gap_after_us"], v["dur_med"]) for k, v in d["per_kernel"].items() if v["n"] == 28}
        print("probe", sys.argv[2], "bal", sys.argv[3], "step_us", d["step_us"], pk)
PY
done
