# Round 3 (session 3): HEAD evidence — flash bench at the adopted parts policy, GPU tier, smoke, driver bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py --lens 1024,2048,4096,8192 > gpurun_out/r3c_final_flash.log 2>&1 || { tail -30 gpurun_out/r3c_final_flash.log; exit 1; }
grep '^{' gpurun_out/r3c_final_flash.log | cut -c1-100
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3c_final_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r3c_final_tests.log; exit 1; }
tail -1 gpurun_out/r3c_final_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3c_final_smoke.log 2>&1 || { tail -30 gpurun_out/r3c_final_smoke.log; exit 1; }
tail -1 gpurun_out/r3c_final_smoke.log | cut -c1-160
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3c_final_bench.log 2>&1 || { tail -30 gpurun_out/r3c_final_bench.log; exit 1; }
tail -1 gpurun_out/r3c_final_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bf16', {k: d[k] for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','timed_engine_idle_ms','timed_prefill_steps')})"
timeout -k 10 500 python -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 512 2048 4096 --chunk 4096 > gpurun_out/r3c_final_ttft_llama.log 2>&1 || { tail -30 gpurun_out/r3c_final_ttft_llama.log; exit 1; }
grep '^{' gpurun_out/r3c_final_ttft_llama.log | cut -c1-200
