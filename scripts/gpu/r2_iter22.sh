set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
VGATE_FUSE_ATTN_O=1 timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r2_tl_fused.log 2>&1 || { tail -30 gpurun_out/r2_tl_fused.log; exit 1; }
grep attn_o_roles gpurun_out/r2_tl_fused.log | head -8
