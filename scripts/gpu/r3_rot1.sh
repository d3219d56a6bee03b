# Round 3: block-rotated k-ranges (activation hot-spot hypothesis): tests, bf16 step A/B, AWQ (lds, rotated loader) A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "rotation or awq_lds or register_groups" > gpurun_out/r3_rot1_tests.log 2>&1 || { tail -40 gpurun_out/r3_rot1_tests.log; exit 1; }
tail -2 gpurun_out/r3_rot1_tests.log
for i in 1 2; do
for r in 0 1; do
  VGATE_DEC_ROT=$r timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only > gpurun_out/r3_rot1_r${r}_$i.log 2>&1 || { tail -30 gpurun_out/r3_rot1_r${r}_$i.log; exit 1; }
  echo "bf16 rot=$r run $i: $(grep -v '^\[' gpurun_out/r3_rot1_r${r}_$i.log | grep us | tr '\n' ' ')"
done
done
for b in 0 1; do
  VGATE_AWQ_LDS=$b timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only --quantization awq > gpurun_out/r3_rot1_awq$b.log 2>&1 || { tail -30 gpurun_out/r3_rot1_awq$b.log; exit 1; }
  echo "awq_lds=$b (rotated loader): $(grep -v '^\[' gpurun_out/r3_rot1_awq$b.log | grep us | tr '\n' ' ')"
done
VGATE_DEC_ROT=1 timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r3_rot1_timeline.log 2>&1 || { tail -30 gpurun_out/r3_rot1_timeline.log; exit 1; }
python - gpurun_out/r3_rot1_timeline.log <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith('{"batch"'):
        d = json.loads(ln)
        print("rot=1 step_us", d["step_us"], {k: (v["avg_span_us"], v["avg_gap_after_us"], v["dur_med"]) for k, v in d["per_kernel"].items() if v["n"] >= 28})
PY
