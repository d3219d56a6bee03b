set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u benchmarks/attn_phases.py > gpurun_out/r2_attn_phases11.log 2>&1 || { tail -20 gpurun_out/r2_attn_phases11.log; exit 1; }
grep ctx gpurun_out/r2_attn_phases11.log
