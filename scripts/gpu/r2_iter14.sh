set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u benchmarks/awq_phases.py > gpurun_out/r2_awq_phases14.log 2>&1 || { tail -20 gpurun_out/r2_awq_phases14.log; exit 1; }
grep shape gpurun_out/r2_awq_phases14.log
