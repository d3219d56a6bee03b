# Round 3: flash prefill with the VALU trimmed (scalar DMA descriptors, v_max3 without canonicalisation)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or prefill or attention" > gpurun_out/r3_flash9_tests.log 2>&1 || { tail -40 gpurun_out/r3_flash9_tests.log; exit 1; }
tail -1 gpurun_out/r3_flash9_tests.log
timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py > gpurun_out/r3_flash9.log 2>&1 || { tail -30 gpurun_out/r3_flash9.log; exit 1; }
grep '{' gpurun_out/r3_flash9.log
