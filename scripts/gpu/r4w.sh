# Round 4: 224 x 160 prefill tile: correctness, mid-M sweep vs the other tiles, prefill-step timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "224x160" > gpurun_out/r4w_tests.log 2>&1 || { tail -40 gpurun_out/r4w_tests.log; exit 1; }
tail -3 gpurun_out/r4w_tests.log
timeout -k 10 300 python -u benchmarks/prefill_tile_sweep.py --ms 384,448,512,1024 --tiles 0,1024,1281,641,2240 --sks 0,2,3 > gpurun_out/r4w_sweep.log 2>&1 || { tail -30 gpurun_out/r4w_sweep.log; exit 1; }
grep gate_up gpurun_out/r4w_sweep.log
timeout -k 10 400 python -u benchmarks/timeline.py --prefill --batch 8 --ctx 50 > gpurun_out/r4w_prefill_timeline.log 2>&1 || { tail -30 gpurun_out/r4w_prefill_timeline.log; exit 1; }
head -c 1500 gpurun_out/r4w_prefill_timeline.log
