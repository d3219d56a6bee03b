# ad-hoc GPU batch (the current experiment); see run.sh for the standing tasks
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu \
  -k "all_epilogues and (1027 or 771)" > gpurun_out/sp1_tests.log 2>&1 || { tail -30 gpurun_out/sp1_tests.log; exit 1; }
tail -1 gpurun_out/sp1_tests.log
for code in 1024 1027 768 771; do
  timeout -k 10 120 python3 -u benchmarks/probes/gemm_pmc_probe.py --code $code >> gpurun_out/sp1_probe.log 2>&1 || { tail -20 gpurun_out/sp1_probe.log; exit 1; }
done
for code in 1024 1027; do
  timeout -k 10 120 python3 -u benchmarks/probes/gemm_pmc_probe.py --code $code --N 6144 >> gpurun_out/sp1_probe.log 2>&1 || { tail -20 gpurun_out/sp1_probe.log; exit 1; }
done
cat gpurun_out/sp1_probe.log
timeout -k 10 300 python -u benchmarks/probes/prefill_cold_sweep.py --model llama8b --ms 2048 --only 1024,1027,768,771 --norm > gpurun_out/sp1_sweep_llama.log 2>&1 || { tail -30 gpurun_out/sp1_sweep_llama.log; exit 1; }
timeout -k 10 300 python -u benchmarks/probes/prefill_cold_sweep.py --model qwen --ms 448,2048 --only 1024,1027,768,771 --norm > gpurun_out/sp1_sweep_qwen.log 2>&1 || { tail -30 gpurun_out/sp1_sweep_qwen.log; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/sp1_sweep_llama.log", "gpurun_out/sp1_sweep_qwen.log"):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); a = d["all"]
            print(d["shape"], d["M"], {k: a[k] for k in a if k.split("/")[0] in ("1024", "1027", "768", "771")})
PY
