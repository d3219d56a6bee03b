# Round 3: flash prefill with the engine's tile order in the bench: ring stages 2 / 4
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 2 4; do
  VGATE_FLASH_NST=$n timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py > gpurun_out/r3_flash7_n$n.log 2>&1 || { tail -30 gpurun_out/r3_flash7_n$n.log; exit 1; }
  echo "NST=$n"; grep '{' gpurun_out/r3_flash7_n$n.log
done
VGATE_FLASH_CT=2 timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py > gpurun_out/r3_flash7_ct2.log 2>&1 || { tail -30 gpurun_out/r3_flash7_ct2.log; exit 1; }
echo "NST=2 CT=2"; grep '{' gpurun_out/r3_flash7_ct2.log | grep -v llama3_8b
