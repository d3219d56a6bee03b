set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u benchmarks/prefill_tile_sweep.py --ms 256,384,512,1024 > gpurun_out/r2b_ptile.log 2>&1 || { tail -30 gpurun_out/r2b_ptile.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r2b_ptile.log"):
    if l.startswith("{"):
        d = json.loads(l); print(d["proj"], d["M"], "lib", d["hipblaslt_us"], "auto", d["auto_us"], "best", d["best"], d["best_us"])
PY
