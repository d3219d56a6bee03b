# Round 4: AWQ wide kernel with the hand-off's sums of squares requested beside the DMA pieces: tests + same-box AWQ step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "awq" > gpurun_out/r4ak_tests.log 2>&1 || { tail -40 gpurun_out/r4ak_tests.log; exit 1; }
tail -1 gpurun_out/r4ak_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "awq" > gpurun_out/r4ak_engine.log 2>&1 || { tail -40 gpurun_out/r4ak_engine.log; exit 1; }
tail -1 gpurun_out/r4ak_engine.log
for i in 1 2; do
  (cd ab_old && timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --quantization awq --baseline-only > ../gpurun_out/r4ak_old_$i.log 2>&1) || { tail -20 gpurun_out/r4ak_old_$i.log; exit 1; }
  echo "old $i"; grep '^{' gpurun_out/r4ak_old_$i.log
  timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --quantization awq --baseline-only > gpurun_out/r4ak_new_$i.log 2>&1 || { tail -20 gpurun_out/r4ak_new_$i.log; exit 1; }
  echo "new $i"; grep '^{' gpurun_out/r4ak_new_$i.log
done
