# Round 3: software-pipelined flash loop (VGATE_FLASH_SWP=1) vs the plain 2-stage loop
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
VGATE_FLASH_SWP=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash" > gpurun_out/r3_flash8_tests.log 2>&1 || { tail -40 gpurun_out/r3_flash8_tests.log; exit 1; }
tail -1 gpurun_out/r3_flash8_tests.log
for swp in 1 0; do
  VGATE_FLASH_SWP=$swp timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py > gpurun_out/r3_flash8_s$swp.log 2>&1 || { tail -30 gpurun_out/r3_flash8_s$swp.log; exit 1; }
  echo "SWP=$swp"; grep '{' gpurun_out/r3_flash8_s$swp.log
done
