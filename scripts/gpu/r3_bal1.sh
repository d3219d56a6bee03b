# Round 3, call 3: balanced decode GEMM (gate_up) correctness, then step-time A/B and timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "balanced or register_groups or gemm_silu" > gpurun_out/r3_bal1_tests.log 2>&1 || { tail -40 gpurun_out/r3_bal1_tests.log; exit 1; }
tail -2 gpurun_out/r3_bal1_tests.log
for i in 1 2; do
for b in 0 1; do
  VGATE_DEC_BAL=$b timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only > gpurun_out/r3_bal1_b${b}_$i.log 2>&1 || { tail -30 gpurun_out/r3_bal1_b${b}_$i.log; exit 1; }
  echo "bal=$b run $i: $(grep -v '^\[' gpurun_out/r3_bal1_b${b}_$i.log | grep us | tr '\n' ' ')"
done
done
VGATE_DEC_BAL=1 timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r3_bal1_timeline.log 2>&1 || { tail -30 gpurun_out/r3_bal1_timeline.log; exit 1; }
grep step_us gpurun_out/r3_bal1_timeline.log | cut -c1-900
