# Round 3 (session 3): flash ring stages (VGATE_FLASH_NST 2 / 4) and lazy rescale (VGATE_FLASH_LAZY 1 / 0) with the split
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "NST=4" "LAZY=0" "NST=2"; do
env VGATE_FLASH_$cfg timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py --lens 1024,2048,4096 > gpurun_out/r3c_flashenv_$cfg.log 2>&1 || { tail -30 gpurun_out/r3c_flashenv_$cfg.log; exit 1; }
echo "$cfg"; grep '^{' gpurun_out/r3c_flashenv_$cfg.log | cut -c1-100
done
