set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 2048 4096 --chunk 4096 > gpurun_out/r2_ttft18.log 2>&1 || { tail -20 gpurun_out/r2_ttft18.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r2_ttft18.log | tail -4
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof_ttft -o run -- python3 benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 2048 --chunk 4096 > gpurun_out/r2_ttft18_prof.log 2>&1 || { tail -20 gpurun_out/r2_ttft18_prof.log; exit 1; }
python benchmarks/prof_summary.py $(ls /tmp/prof_ttft/*.db /tmp/prof_ttft/*/*.db 2>/dev/null | head -1) --top 25 > gpurun_out/r2_ttft18_kernels.txt 2>&1 || true
head -22 gpurun_out/r2_ttft18_kernels.txt
