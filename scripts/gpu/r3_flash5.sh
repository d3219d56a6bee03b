# Round 3: flash prefill v5 (4-stage LDS-DMA ring, 64-query Llama blocks)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "prefill or attention or engine or flash" > gpurun_out/r3_flash5_tests.log 2>&1 || { tail -40 gpurun_out/r3_flash5_tests.log; exit 1; }
tail -2 gpurun_out/r3_flash5_tests.log
timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py > gpurun_out/r3_flash5_bench.log 2>&1 || { tail -30 gpurun_out/r3_flash5_bench.log; exit 1; }
grep '{' gpurun_out/r3_flash5_bench.log
VGATE_FLASH_CT=2 timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py > gpurun_out/r3_flash5_bench_ct2.log 2>&1 || { tail -30 gpurun_out/r3_flash5_bench_ct2.log; exit 1; }
echo "CT=2 forced:"; grep '{' gpurun_out/r3_flash5_bench_ct2.log | grep -v llama3_8b
timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only > gpurun_out/r3_flash5_dec.log 2>&1 || { tail -30 gpurun_out/r3_flash5_dec.log; exit 1; }
grep -v '^\[' gpurun_out/r3_flash5_dec.log | grep us | tr '\n' ' '
