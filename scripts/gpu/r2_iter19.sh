set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "prefill" --timeout 200 --timeout-method thread > gpurun_out/r2_kern19.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/r2_kern19.log; exit 1; }
tail -1 gpurun_out/r2_kern19.log
timeout -k 10 400 python -u benchmarks/prefill_gemm_bench.py --ms 512,1024,2048,4096 --models llama8b,qwen > gpurun_out/r2_pgemm19.log 2>&1 || { tail -20 gpurun_out/r2_pgemm19.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r2_pgemm19.log"):
    if l.startswith("{"):
        d = json.loads(l)
        if "model" in d: print(d["model"], d["proj"], d["M"], d["ours_tflops"], d["hipblaslt_tflops"], d["ratio_vs_lib"], d["rel_err"])
        else: print(d)
PY
true
true
