# Round 4 final: scenario report (benchmarks/run_report.py --engine native) at the last commit
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u benchmarks/run_report.py --engine native --out gpurun_out/r4ao_report > gpurun_out/r4ao_report.log 2>&1 || { tail -30 gpurun_out/r4ao_report.log; exit 1; }
tail -12 gpurun_out/r4ao_report.log | cut -c1-200
