# Round 3 (session 2): flash prefill column tiles per wave for the 2-KV-head Qwen layout (CT=1 default vs VGATE_FLASH_CT=2), 1k-8k tokens
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for ct in 0 2; do
VGATE_FLASH_CT=$ct timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py --lens 1024,2048,4096,8192 > gpurun_out/r3b_flashct_$ct.log 2>&1 || { tail -30 gpurun_out/r3b_flashct_$ct.log; exit 1; }
echo "CT=$ct"; grep '^{' gpurun_out/r3b_flashct_$ct.log | grep qwen | cut -c1-160
done
