# Round 5: bf16 RMSNorm sum-of-squares hand-off (o/down epilogues -> qkv/gate_up row scale): GPU tier, timeline, driver bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r5g_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5g_tests.log; exit 1; }
tail -2 gpurun_out/r5g_tests.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r5g_timeline.log 2>&1 || { tail -30 gpurun_out/r5g_timeline.log; exit 1; }
grep '"step_us"' gpurun_out/r5g_timeline.log | cut -c1-200
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5g_bench.log 2>&1 || { tail -30 gpurun_out/r5g_bench.log; exit 1; }
tail -1 gpurun_out/r5g_bench.log | cut -c1-400
mkdir -p build && hipcc --offload-arch=gfx950 -O3 -I csrc/kernels -o build/decode_gemm_anatomy benchmarks/probes/decode_gemm_anatomy.hip
timeout -k 10 240 ./build/decode_gemm_anatomy > gpurun_out/r5h_anatomy.log 2>&1 || { tail -20 gpurun_out/r5h_anatomy.log; exit 1; }
cat gpurun_out/r5h_anatomy.log
