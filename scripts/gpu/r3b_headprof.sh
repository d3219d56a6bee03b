# Round 3 (session 2): rocprofv3 kernel trace of the driver bench command at HEAD, summarised on the box (the db is not kept)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r3b_headprof -o bench -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3b_headprof_bench.log 2>&1 || { tail -30 gpurun_out/r3b_headprof_bench.log; exit 1; }
tail -1 gpurun_out/r3b_headprof_bench.log | cut -c1-300
python3 benchmarks/prof_summary.py /tmp/r3b_headprof/bench_results.db --top 45 > gpurun_out/r3b_headprof_kernels.txt
head -30 gpurun_out/r3b_headprof_kernels.txt | cut -c1-150
