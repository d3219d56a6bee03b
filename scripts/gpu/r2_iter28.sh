set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "prefill_lds_gemm" --timeout 120 --timeout-method thread > gpurun_out/r2_pt28.log 2>&1 || { echo T_FAIL; tail -40 gpurun_out/r2_pt28.log; exit 1; }
tail -1 gpurun_out/r2_pt28.log
for bn in 0 512; do
timeout -k 10 400 python -u benchmarks/prefill_gemm_bench.py --ms 1024,2048,4096 --models llama8b,qwen --bn $bn > gpurun_out/r2_pg28_$bn.log 2>&1 || { tail -20 gpurun_out/r2_pg28_$bn.log; exit 1; }
echo "== bn=$bn"
python - $bn <<'PY'
import json, sys
for l in open(f"gpurun_out/r2_pg28_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        if "model" in d: print(d["model"], d["proj"], d["M"], d["ours_tflops"], d["hipblaslt_tflops"], d["ratio_vs_lib"], d["rel_err"])
        else: print(d)
PY
done
