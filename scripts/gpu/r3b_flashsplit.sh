# Round 3 (session 2): flash prefill causal K split (two halves met through the GEMM workspace) —
# numerics (flash GPU test) then throughput split on vs off, 1k-8k tokens, and TTFT at 2048
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attention" > gpurun_out/r3b_flashsplit_test.log 2>&1 || { tail -40 gpurun_out/r3b_flashsplit_test.log; exit 1; }
tail -3 gpurun_out/r3b_flashsplit_test.log
for sp in 1 0; do
VGATE_FLASH_SPLIT=$sp timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py --lens 1024,2048,4096,8192 > gpurun_out/r3b_flashsplit_$sp.log 2>&1 || { tail -30 gpurun_out/r3b_flashsplit_$sp.log; exit 1; }
echo "SPLIT=$sp"; grep '^{' gpurun_out/r3b_flashsplit_$sp.log | cut -c1-200
done
