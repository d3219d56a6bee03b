# ad-hoc GPU batch (the current experiment); see run.sh for the standing tasks
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu \
  -k "prefill or persistent_k_split" > gpurun_out/sk4_tests.log 2>&1 || { tail -30 gpurun_out/sk4_tests.log; exit 1; }
tail -2 gpurun_out/sk4_tests.log
timeout -k 10 300 python -u benchmarks/probes/prefill_cold_sweep.py --model llama8b --ms 2048 --only 1024,1025,768,769 --norm > gpurun_out/sk4_sweep_llama_norm.log 2>&1 || { tail -30 gpurun_out/sk4_sweep_llama_norm.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/sk4_sweep_llama_norm.log"):
    if l.startswith("{"):
        d = json.loads(l); a = d["all"]
        print(d["shape"], d["M"], "best_cold", d["best_cold"], "best_warm", d["best_warm"], "blas", d["hipblaslt"], {k: a[k] for k in a if k in ("1024/0", "1025/0", "768/0", "769/0")})
PY
timeout -k 10 400 python -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 512 2048 4096 > gpurun_out/sk4_ttft.log 2>&1 || { tail -30 gpurun_out/sk4_ttft.log; exit 1; }
grep '^{' gpurun_out/sk4_ttft.log | tail -3
timeout -k 10 400 python -u benchmarks/timeline.py --model meta-llama/Meta-Llama-3-8B-Instruct --prefill --batch 1 --ctx 2000 > gpurun_out/sk4_llama_ptimeline.log 2>&1 || { tail -30 gpurun_out/sk4_llama_ptimeline.log; exit 1; }
grep -m1 -o '"launches": [0-9]*, "step_us": [0-9.]*' gpurun_out/sk4_llama_ptimeline.log
timeout -k 10 300 python -u benchmarks/timeline.py --prefill --batch 8 --ctx 50 > gpurun_out/sk4_qwen_ptimeline.log 2>&1 || { tail -30 gpurun_out/sk4_qwen_ptimeline.log; exit 1; }
grep -m1 -o '"launches": [0-9]*, "step_us": [0-9.]*' gpurun_out/sk4_qwen_ptimeline.log
