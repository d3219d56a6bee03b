# Round 4: 4-deep-ring 128-row prefill tiles (numerics + mid-M sweep); decode timeline through the captured graph; driver bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -k prefill_lds_gemm -x -q --timeout 120 --timeout-method thread > gpurun_out/r4g_tiles_test.log 2>&1 || { echo TILE_TEST_FAIL; tail -60 gpurun_out/r4g_tiles_test.log; exit 1; }
tail -1 gpurun_out/r4g_tiles_test.log
timeout -k 10 300 python -u benchmarks/prefill_tile_sweep.py --ms 128,256,384,512 --model qwen --tiles 0,64,128,768,1280,1281,640,641 --sks 0,2,3 > gpurun_out/r4g_sweep_qwen.log 2>&1 || { tail -30 gpurun_out/r4g_sweep_qwen.log; exit 1; }
cut -c1-200 gpurun_out/r4g_sweep_qwen.log
timeout -k 10 300 python -u benchmarks/prefill_tile_sweep.py --ms 256,384,512 --model llama8b --tiles 0,64,128,768,1280,1281,640,641 --sks 0,2,3 > gpurun_out/r4g_sweep_llama.log 2>&1 || { tail -30 gpurun_out/r4g_sweep_llama.log; exit 1; }
cut -c1-200 gpurun_out/r4g_sweep_llama.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 --replays 3 > gpurun_out/r4g_timeline.log 2>&1 || { tail -30 gpurun_out/r4g_timeline.log; exit 1; }
grep '"launches"' gpurun_out/r4g_timeline.log | cut -c1-400
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4g_bench.log 2>&1 || { tail -30 gpurun_out/r4g_bench.log; exit 1; }
tail -1 gpurun_out/r4g_bench.log | cut -c1-900
