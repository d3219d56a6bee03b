set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u benchmarks/qa_phases.py --oproj >> gpurun_out/r5ae_ph.log 2>&1 || { tail -30 gpurun_out/r5ae_ph.log; exit 1; }
grep '^{' gpurun_out/r5ae_ph.log
