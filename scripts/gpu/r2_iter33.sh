set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "prefill_lds_gemm" --timeout 120 --timeout-method thread > gpurun_out/r2_pt33.log 2>&1 || { echo T_FAIL; tail -40 gpurun_out/r2_pt33.log; exit 1; }
tail -1 gpurun_out/r2_pt33.log
for bn in 0; do
timeout -k 10 400 python -u benchmarks/prefill_gemm_bench.py --ms 512,1024,2048,4096 --models llama8b,qwen,llama70b_tp8 --bn $bn > gpurun_out/r2_pg33_$bn.log 2>&1 || { tail -20 gpurun_out/r2_pg33_$bn.log; exit 1; }
echo "== bn=$bn $(python - $bn <<'PY'
import json, sys
r = []
for l in open(f"gpurun_out/r2_pg33_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        if "model" in d: r.append(f"{d['model'][:2]}{d['proj']}{d['M']}:{d['ours_tflops']:.0f}/{d['hipblaslt_tflops']:.0f}")
        else: r.append(str(d["summary"]["geomean_ratio_vs_hipblaslt"]))
print(" ".join(r))
PY
)"
done
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 2048 4096 --chunk 4096 > gpurun_out/r2_ttft33.log 2>&1 || { tail -20 gpurun_out/r2_ttft33.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r2_ttft33.log | tail -4
