# Round 3: flash prefill A/B: ring stages (VGATE_FLASH_NST) x lazy rescale (VGATE_FLASH_LAZY)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash" > gpurun_out/r3_flash6_tests.log 2>&1 || { tail -40 gpurun_out/r3_flash6_tests.log; exit 1; }
tail -1 gpurun_out/r3_flash6_tests.log
for cfg in "2 1" "2 0" "3 1" "4 1"; do
  set -- $cfg
  VGATE_FLASH_NST=$1 VGATE_FLASH_LAZY=$2 timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py > gpurun_out/r3_flash6_n$1_l$2.log 2>&1 || { tail -30 gpurun_out/r3_flash6_n$1_l$2.log; exit 1; }
  echo "NST=$1 LAZY=$2"; grep '{' gpurun_out/r3_flash6_n$1_l$2.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('  ', d['layout'], d['S'], d['flash_us'], d['flash_tflops'])"
done
