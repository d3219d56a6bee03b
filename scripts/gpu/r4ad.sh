# Round 4: single-launch granule sampler: kernel + engine tests, decode-step A/B (pass kernels vs single launch), timeline, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sample" > gpurun_out/r4ad_tests.log 2>&1 || { tail -40 gpurun_out/r4ad_tests.log; exit 1; }
tail -1 gpurun_out/r4ad_tests.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py > gpurun_out/r4ad_engine.log 2>&1 || { tail -40 gpurun_out/r4ad_engine.log; exit 1; }
tail -1 gpurun_out/r4ad_engine.log
for i in 1 2; do
  VGATE_SAMPLE_SINGLE=0 timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only > gpurun_out/r4ad_pass_$i.log 2>&1 || { tail -20 gpurun_out/r4ad_pass_$i.log; exit 1; }
  echo "pass kernels $i"; grep '^{' gpurun_out/r4ad_pass_$i.log
  timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only > gpurun_out/r4ad_single_$i.log 2>&1 || { tail -20 gpurun_out/r4ad_single_$i.log; exit 1; }
  echo "single launch $i"; grep '^{' gpurun_out/r4ad_single_$i.log
done
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r4ad_timeline.log 2>&1 || { tail -30 gpurun_out/r4ad_timeline.log; exit 1; }
head -c 400 gpurun_out/r4ad_timeline.log; echo
grep -o '"sample_gran[^}]*}' gpurun_out/r4ad_timeline.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4ad_bench.log 2>&1 || { tail -30 gpurun_out/r4ad_bench.log; exit 1; }
grep '^{' gpurun_out/r4ad_bench.log | cut -c1-400
