# Round 4: single-launch sampler without the exit ticket (epoch advanced by plain stores): tests, probe, step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sample" > gpurun_out/r4af_tests.log 2>&1 || { tail -40 gpurun_out/r4af_tests.log; exit 1; }
tail -1 gpurun_out/r4af_tests.log
timeout -k 10 300 python -u benchmarks/sampler_probe.py > gpurun_out/r4af_probe.log 2>&1 || { tail -30 gpurun_out/r4af_probe.log; exit 1; }
grep '^{' gpurun_out/r4af_probe.log | head -1 | cut -c300-600
timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only > gpurun_out/r4af_step.log 2>&1 || { tail -20 gpurun_out/r4af_step.log; exit 1; }
grep '^{' gpurun_out/r4af_step.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r4af_timeline.log 2>&1 || { tail -30 gpurun_out/r4af_timeline.log; exit 1; }
head -c 300 gpurun_out/r4af_timeline.log; echo
grep -o '"sample_gran[^}]*}' gpurun_out/r4af_timeline.log
