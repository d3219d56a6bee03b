set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf /tmp/prof_awq35
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_awq35 -o run -- python3 bench.py --gpus 1 --steps 10 --warmup 3 --quantization awq --security > gpurun_out/r2_prof35_awq.log 2>&1 || { tail -20 gpurun_out/r2_prof35_awq.log; exit 1; }
python benchmarks/prof_summary.py $(ls /tmp/prof_awq35/*.db /tmp/prof_awq35/*/*.db 2>/dev/null | head -1) --top 16 > gpurun_out/r2_awq35_kernels.txt 2>&1 || true
head -14 gpurun_out/r2_awq35_kernels.txt | cut -c1-150
