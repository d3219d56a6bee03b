# Round 4: in-engine decode decomposition sweep for gate_up / down with the granule split-K combine (whole-step graph replays)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --kinds gate_up,down > gpurun_out/r4s_sweep.log 2>&1 || { tail -30 gpurun_out/r4s_sweep.log; exit 1; }
grep '^{' gpurun_out/r4s_sweep.log
