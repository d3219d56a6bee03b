set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u benchmarks/decode_sweep.py --kinds down,qkv,o --ctx 100 > gpurun_out/r2b_dsweep.log 2>&1 || { tail -30 gpurun_out/r2b_dsweep.log; exit 1; }
grep "^{" gpurun_out/r2b_dsweep.log
