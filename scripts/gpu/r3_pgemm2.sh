# Round 3: prefill GEMM vs hipBLASLt with the engine's start-up tuned decomposition
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u benchmarks/prefill_gemm_bench.py --ms 512,1024,2048,4096 --tuned --iters 10 > gpurun_out/r3_pgemm2.log 2>&1 || { tail -30 gpurun_out/r3_pgemm2.log; exit 1; }
python3 - gpurun_out/r3_pgemm2.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        if 'summary' in d: print(d); continue
        print(d['model'], d['proj'], d['M'], d['ours_tflops'], d['hipblaslt_tflops'], d['ratio_vs_lib'], d['plan'])
PY
