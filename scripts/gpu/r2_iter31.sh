set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 2048 4096 --chunk 4096 > gpurun_out/r2_ttft31.log 2>&1 || { tail -20 gpurun_out/r2_ttft31.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r2_ttft31.log | tail -4
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof_ttft -o run -- python3 benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 2048 --chunk 4096 > gpurun_out/r2_ttft31_prof.log 2>&1 || { tail -20 gpurun_out/r2_ttft31_prof.log; exit 1; }
python benchmarks/prof_summary.py $(ls /tmp/prof_ttft/*.db /tmp/prof_ttft/*/*.db 2>/dev/null | head -1) --top 25 > gpurun_out/r2_ttft31_kernels.txt 2>&1 || true
head -22 gpurun_out/r2_ttft31_kernels.txt
timeout -k 10 300 python -u benchmarks/ttft_probe.py --model Qwen/Qwen2.5-1.5B-Instruct --lens 512 2048 4096 --chunk 4096 > gpurun_out/r2_ttft31_qwen.log 2>&1 || { tail -20 gpurun_out/r2_ttft31_qwen.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r2_ttft31_qwen.log | tail -4
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2_gpu31.log 2>&1 || { echo GPU_FAIL; tail -40 gpurun_out/r2_gpu31.log; exit 1; }
tail -1 gpurun_out/r2_gpu31.log
