# ad-hoc GPU batch: the folded norm's cost on the serving-size prefill tiles (Qwen2.5-1.5B, 448 rows)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for n in "" "--norm"; do
timeout -k 10 300 python -u benchmarks/probes/prefill_cold_sweep.py --model qwen --ms 448 --only 2560,2561,1281,128 $n > gpurun_out/nc_sweep$n.log 2>&1 || { tail -30 gpurun_out/nc_sweep$n.log; exit 1; }
python3 - "gpurun_out/nc_sweep$n.log" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); a = d["all"]
        print(sys.argv[1][-12:], d["shape"], d["M"], {k: a[k] for k in a if k in ("2560/0", "2561/0", "1281/0", "128/0")})
PY
done
