# Round 5: kx int4 kernel, multi-tile GROUP blocks: numerics, per-shape (waves, slices) sweep, AWQ timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "awq" > gpurun_out/r5l_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5l_tests.log; exit 1; }
tail -2 gpurun_out/r5l_tests.log
timeout -k 10 300 python -u benchmarks/awq_sweep.py > gpurun_out/r5l_sweep.log 2>&1 || { tail -30 gpurun_out/r5l_sweep.log; exit 1; }
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 --quantization awq > gpurun_out/r5l_timeline.log 2>&1 || { tail -30 gpurun_out/r5l_timeline.log; exit 1; }
grep '"step_us"' gpurun_out/r5l_timeline.log | cut -c1-120
