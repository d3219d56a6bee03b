# ad-hoc GPU batch (the current experiment); see run.sh for the standing tasks
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu \
  -k "prefill or persistent_k_split" > gpurun_out/nc2_tests.log 2>&1 || { tail -30 gpurun_out/nc2_tests.log; exit 1; }
tail -1 gpurun_out/nc2_tests.log
timeout -k 10 300 python -u benchmarks/probes/prefill_cold_sweep.py --model qwen --ms 448 --only 2560,2561,1281,128 --norm > gpurun_out/nc2_sweep_norm.log 2>&1 || { tail -30 gpurun_out/nc2_sweep_norm.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/nc2_sweep_norm.log"):
    if l.startswith("{"):
        d = json.loads(l); a = d["all"]
        print("norm", d["shape"], d["M"], {k: a[k] for k in a if k in ("2560/0", "2561/0", "1281/0", "128/0")})
PY
bash scripts/gpu/run.sh nc2 bench ptimeline
