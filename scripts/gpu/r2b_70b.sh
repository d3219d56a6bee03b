set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u benchmarks/bench_endpoint.py --model meta-llama/Meta-Llama-3-70B --rounds 5 > gpurun_out/r2b_70b.log 2>&1 || { tail -30 gpurun_out/r2b_70b.log; exit 1; }
tail -3 gpurun_out/r2b_70b.log | cut -c1-600
