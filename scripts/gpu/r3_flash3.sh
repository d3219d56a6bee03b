# Round 3: flash prefill with the block table staged in LDS, folded into the unified attention launch
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "prefill or attention or engine" > gpurun_out/r3_flash3_tests.log 2>&1 || { tail -40 gpurun_out/r3_flash3_tests.log; exit 1; }
tail -2 gpurun_out/r3_flash3_tests.log
timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py > gpurun_out/r3_flash3_bench.log 2>&1 || { tail -30 gpurun_out/r3_flash3_bench.log; exit 1; }
grep '{' gpurun_out/r3_flash3_bench.log
timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only > gpurun_out/r3_flash3_dec.log 2>&1 || { tail -30 gpurun_out/r3_flash3_dec.log; exit 1; }
grep -v '^\[' gpurun_out/r3_flash3_dec.log | grep us | tr '\n' ' '
