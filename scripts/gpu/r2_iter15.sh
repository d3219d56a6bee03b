set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for pr in 0 1 2 3; do
VGATE_AWQ_PROBE=$pr AWQ_SWEEP_SHAPES=gate_up,down timeout -k 10 200 python -u benchmarks/awq_sweep.py > gpurun_out/r2_awq_probe$pr.log 2>&1 || { tail -20 gpurun_out/r2_awq_probe$pr.log; exit 1; }
echo "PROBE=$pr"; grep shape gpurun_out/r2_awq_probe$pr.log
done
