# Round 4: in-engine AWQ decode decomposition sweep (granule split-K, epilogue prefetch) for qkv / o / down
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --quantization awq --kinds down,qkv,o > gpurun_out/r4t_awq_sweep.log 2>&1 || { tail -30 gpurun_out/r4t_awq_sweep.log; exit 1; }
grep '^{' gpurun_out/r4t_awq_sweep.log
