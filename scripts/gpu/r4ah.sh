# Round 4: single-launch sampler, epoch advanced by segment 0 only: tests + probe + step (same box), ticket-free
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sample" > gpurun_out/r4ah_tests.log 2>&1 || { tail -40 gpurun_out/r4ah_tests.log; exit 1; }
tail -1 gpurun_out/r4ah_tests.log
for m in 1 0 1; do
  VGATE_SAMPLE_SINGLE=$m timeout -k 10 300 python -u benchmarks/sampler_probe.py > gpurun_out/r4ah_probe_$m.log 2>&1 || { tail -30 gpurun_out/r4ah_probe_$m.log; exit 1; }
  echo "single=$m"; grep '^{' gpurun_out/r4ah_probe_$m.log | head -1 | cut -c280-600
done
timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only > gpurun_out/r4ah_step.log 2>&1 || { tail -20 gpurun_out/r4ah_step.log; exit 1; }
grep '^{' gpurun_out/r4ah_step.log
