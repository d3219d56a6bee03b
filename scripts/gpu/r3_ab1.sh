# Round 3, call 2: correctness of the new register-group sizes (GEMM GPU tests), then step-time A/B
# of the decode register-group rule: round-2 rule (VGATE_DEC_U=-1) vs all-in-two-groups (0)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/r3_ab1_tests.log 2>&1 || { tail -40 gpurun_out/r3_ab1_tests.log; exit 1; }
tail -2 gpurun_out/r3_ab1_tests.log
for i in 1 2; do
for u in -1 0; do
  VGATE_DEC_U=$u timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only > gpurun_out/r3_ab1_u${u}_$i.log 2>&1 || { tail -30 gpurun_out/r3_ab1_u${u}_$i.log; exit 1; }
  echo "u=$u run $i: $(grep -v '^\[' gpurun_out/r3_ab1_u${u}_$i.log | grep us | tr '\n' ' ')"
done
done
VGATE_DEC_U=0 timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r3_ab1_timeline.log 2>&1 || { tail -30 gpurun_out/r3_ab1_timeline.log; exit 1; }
grep step_us gpurun_out/r3_ab1_timeline.log | cut -c1-1500
