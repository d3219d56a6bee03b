set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_g1
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_g1 -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/r2b_bench_g1.log 2>&1 || { tail -30 gpurun_out/r2b_bench_g1.log; exit 1; }
DB=$(find gpurun_out/prof_g1 -name "*results.db" | head -1)
python benchmarks/trace_gaps.py $DB --first 12 > gpurun_out/r2b_gaps1.log 2>&1 || { cat gpurun_out/r2b_gaps1.log; exit 1; }
cat gpurun_out/r2b_gaps1.log
tail -1 gpurun_out/r2b_bench_g1.log | cut -c1-300
rm -rf gpurun_out/prof_g1
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r2b_timeline1.log 2>&1 || { tail -30 gpurun_out/r2b_timeline1.log; exit 1; }
tail -5 gpurun_out/r2b_timeline1.log | cut -c1-3000
