# Round 3 (session 3): flash split into up to 4 parts — numerics, A/B parts 4 / 2, Qwen CT=2 with the split,
# then the kernel stats of the Llama-3-8B TTFT probe (2048 / 4096)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attention" > gpurun_out/r3c_flash4_test.log 2>&1 || { tail -40 gpurun_out/r3c_flash4_test.log; exit 1; }
tail -1 gpurun_out/r3c_flash4_test.log
for np in 4 2; do
VGATE_FLASH_PARTS=$np timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py --lens 1024,2048,4096,8192 > gpurun_out/r3c_flash4_p$np.log 2>&1 || { tail -30 gpurun_out/r3c_flash4_p$np.log; exit 1; }
echo "PARTS=$np"; grep '^{' gpurun_out/r3c_flash4_p$np.log | cut -c1-110
done
VGATE_FLASH_CT=2 timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py --lens 1024,2048,4096,8192 > gpurun_out/r3c_flash_ct2split.log 2>&1 || { tail -30 gpurun_out/r3c_flash_ct2split.log; exit 1; }
echo "CT=2 + split"; grep '^{' gpurun_out/r3c_flash_ct2split.log | grep qwen | cut -c1-110
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/ttftprof -o ttft -- python3 -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 2048 4096 --chunk 4096 > gpurun_out/r3c_ttftprof.log 2>&1 || { tail -30 gpurun_out/r3c_ttftprof.log; exit 1; }
grep '^{' gpurun_out/r3c_ttftprof.log
f=$(find /tmp/ttftprof -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/r3c_ttftprof_kernel_stats.csv
head -16 "$f" | cut -c1-160
