# Round 3: AWQ decode with the LDS-shared activation slice: correctness, step A/B, timeline, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "awq" > gpurun_out/r3_awq1_tests.log 2>&1 || { tail -40 gpurun_out/r3_awq1_tests.log; exit 1; }
tail -2 gpurun_out/r3_awq1_tests.log
for i in 1 2; do
for b in 0 1; do
  VGATE_AWQ_LDS=$b timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only --quantization awq > gpurun_out/r3_awq1_l${b}_$i.log 2>&1 || { tail -30 gpurun_out/r3_awq1_l${b}_$i.log; exit 1; }
  echo "awq_lds=$b run $i: $(grep -v '^\[' gpurun_out/r3_awq1_l${b}_$i.log | grep us | tr '\n' ' ')"
done
done
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 --quantization awq > gpurun_out/r3_awq1_timeline.log 2>&1 || { tail -30 gpurun_out/r3_awq1_timeline.log; exit 1; }
python - gpurun_out/r3_awq1_timeline.log <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith('{"batch"'):
        d = json.loads(ln)
        print("step_us", d["step_us"], {k: (v["avg_span_us"], v["avg_gap_after_us"], v["dur_med"]) for k, v in d["per_kernel"].items() if v["n"] >= 28})
PY
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r3_awq1_bench.log 2>&1 || { tail -30 gpurun_out/r3_awq1_bench.log; exit 1; }
tail -1 gpurun_out/r3_awq1_bench.log | cut -c1-400
