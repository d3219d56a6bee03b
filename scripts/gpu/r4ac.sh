# Round 4: the fused TP epilogue as its own instantiations (EPI_BF16_AR): fused / TP tests, same-box A/B of the TP=1 step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_ar_gpu.py > gpurun_out/r4ac_fused_tests.log 2>&1 || { tail -40 gpurun_out/r4ac_fused_tests.log; exit 1; }
tail -1 gpurun_out/r4ac_fused_tests.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tp_gpu.py > gpurun_out/r4ac_tp_tests.log 2>&1 || { tail -40 gpurun_out/r4ac_tp_tests.log; exit 1; }
tail -1 gpurun_out/r4ac_tp_tests.log
for i in 1 2; do
  (cd ab_old && timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only > ../gpurun_out/r4ac_old_$i.log 2>&1) || { tail -20 gpurun_out/r4ac_old_$i.log; exit 1; }
  echo "old $i"; grep '^{' gpurun_out/r4ac_old_$i.log
  timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only > gpurun_out/r4ac_new_$i.log 2>&1 || { tail -20 gpurun_out/r4ac_new_$i.log; exit 1; }
  echo "new $i"; grep '^{' gpurun_out/r4ac_new_$i.log
done
timeout -k 10 400 python -u benchmarks/tp_rank_bench.py --fused-ar > gpurun_out/r4ac_tp8_fused.log 2>&1 || { tail -30 gpurun_out/r4ac_tp8_fused.log; exit 1; }
grep '^{' gpurun_out/r4ac_tp8_fused.log | cut -c1-300
