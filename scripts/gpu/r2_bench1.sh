set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench1.json.log 2>&1 || { tail -20 gpurun_out/r2_bench1.json.log; exit 1; }
tail -1 gpurun_out/r2_bench1.json.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench1 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench1_prof.log 2>&1 || { tail -20 gpurun_out/r2_bench1_prof.log; exit 1; }
python benchmarks/prof_summary.py $(ls gpurun_out/prof_bench1/*.db gpurun_out/prof_bench1/*/*.db 2>/dev/null | head -1) --top 40 > gpurun_out/r2_bench1_kernels.txt 2>&1 || true
head -30 gpurun_out/r2_bench1_kernels.txt
timeout -k 10 200 python -u benchmarks/timeline.py --json gpurun_out/r2_timeline1.json > gpurun_out/r2_timeline1.log 2>&1; head -1 gpurun_out/r2_timeline1.log
