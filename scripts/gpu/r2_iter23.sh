set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof23
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof23 -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/r2_bench23.log 2>&1 || { tail -30 gpurun_out/r2_bench23.log; exit 1; }
DB=$(find gpurun_out/prof23 -name "*results.db" | head -1)
python benchmarks/trace_gaps.py $DB --first 8 > gpurun_out/r2_gaps23.log 2>&1 || { cat gpurun_out/r2_gaps23.log; exit 1; }
cat gpurun_out/r2_gaps23.log
tail -1 gpurun_out/r2_bench23.log | cut -c1-300
rm -rf gpurun_out/prof23
