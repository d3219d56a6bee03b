# Round 4: prefill tile sweep at the TTFT chunk sizes (1024 / 2048 rows) for Llama-3-8B and Qwen2.5-1.5B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u benchmarks/prefill_tile_sweep.py --model llama8b --ms 1024,2048 --tiles 0,768,1024,256,1281 --sks 0,2,3,4 > gpurun_out/r4y_sweep_llama.log 2>&1 || { tail -30 gpurun_out/r4y_sweep_llama.log; exit 1; }
grep '^{' gpurun_out/r4y_sweep_llama.log | cut -c1-200
timeout -k 10 300 python -u benchmarks/prefill_tile_sweep.py --model qwen --ms 1024,2048 --tiles 0,768,1024,256,1281 --sks 0,2,3,4 > gpurun_out/r4y_sweep_qwen.log 2>&1 || { tail -30 gpurun_out/r4y_sweep_qwen.log; exit 1; }
grep '^{' gpurun_out/r4y_sweep_qwen.log | cut -c1-200
