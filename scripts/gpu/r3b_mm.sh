# Round 3 (session 2): medium-M GEMM paths (mixed prefill + decode steps) vs the prefill kernels; AWQ decode sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/medium_m_bench.py > gpurun_out/r3b_mm_qwen.log 2>&1 || { tail -30 gpurun_out/r3b_mm_qwen.log; exit 1; }
python3 - gpurun_out/r3b_mm_qwen.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); print(d["shape"], d["M"], d["default_us"], d["best"], d["best_us"], d["speedup"])
PY
timeout -k 10 600 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --quantization awq --kinds qkv,o,gate_up,down > gpurun_out/r3b_awqsweep.log 2>&1 || { tail -30 gpurun_out/r3b_awqsweep.log; exit 1; }
grep '^{' gpurun_out/r3b_awqsweep.log
