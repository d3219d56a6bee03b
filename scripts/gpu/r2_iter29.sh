set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for sch in 0 1 2; do
timeout -k 10 300 env VGATE_PREFILL_SCHED=$sch python -u -m pytest tests/test_kernels_gpu.py -x -q -k "prefill_lds_gemm and 512" --timeout 120 --timeout-method thread > gpurun_out/r2_pt29.log 2>&1 || { echo T_FAIL $sch; tail -40 gpurun_out/r2_pt29.log; exit 1; }
for bn in 256 512; do
timeout -k 10 400 env VGATE_PREFILL_SCHED=$sch python -u benchmarks/prefill_gemm_bench.py --ms 2048,4096 --models llama8b,qwen --bn $bn > gpurun_out/r2_pg29_${sch}_$bn.log 2>&1 || { tail -20 gpurun_out/r2_pg29_${sch}_$bn.log; exit 1; }
echo "== sched=$sch bn=$bn $(python - $sch $bn <<'PY'
import json, sys
r = []
for l in open(f"gpurun_out/r2_pg29_{sys.argv[1]}_{sys.argv[2]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        if "model" in d: r.append(f"{d['model'][:2]}{d['proj']}{d['M']}:{d['ours_tflops']:.0f}")
        else: r.append(str(d["summary"]["geomean_ratio_vs_hipblaslt"]))
print(" ".join(r))
PY
)"
done
done
