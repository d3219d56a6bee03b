# ad-hoc GPU batch (the current experiment); see run.sh for the standing tasks
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu \
  -k "prefill or persistent_k_split" > gpurun_out/sk9_tests.log 2>&1 || { tail -30 gpurun_out/sk9_tests.log; exit 1; }
tail -1 gpurun_out/sk9_tests.log
timeout -k 10 400 python -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 512 2048 4096 > gpurun_out/sk9_ttft.log 2>&1 || { tail -30 gpurun_out/sk9_ttft.log; exit 1; }
grep '^{' gpurun_out/sk9_ttft.log | tail -3
timeout -k 10 400 python -u benchmarks/ttft_probe.py --lens 512 2048 4096 > gpurun_out/sk9_ttft_qwen.log 2>&1 || { tail -30 gpurun_out/sk9_ttft_qwen.log; exit 1; }
grep '^{' gpurun_out/sk9_ttft_qwen.log | tail -3
