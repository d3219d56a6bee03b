set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_bf16 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_prof17_bf16.log 2>&1 || { tail -20 gpurun_out/r2_prof17_bf16.log; exit 1; }
grep '^{' gpurun_out/r2_prof17_bf16.log | tail -1 | cut -c1-400
python benchmarks/prof_summary.py $(ls /tmp/prof_bf16/*.db /tmp/prof_bf16/*/*.db 2>/dev/null | head -1) --top 30 > gpurun_out/r2_prof17_bf16_kernels.txt 2>&1 || true
head -16 gpurun_out/r2_prof17_bf16_kernels.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_awq -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r2_prof17_awq.log 2>&1 || { tail -20 gpurun_out/r2_prof17_awq.log; exit 1; }
python benchmarks/prof_summary.py $(ls /tmp/prof_awq/*.db /tmp/prof_awq/*/*.db 2>/dev/null | head -1) --top 30 > gpurun_out/r2_prof17_awq_kernels.txt 2>&1 || true
head -16 gpurun_out/r2_prof17_awq_kernels.txt
