# A/B: copies through SDMA engines (default) vs blit kernels on the compute queue (HSA_ENABLE_SDMA=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','engine_avg_step_ms')})"; }
b() {
  tag=$1; shift
  timeout -k 10 300 env "$@" python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2b_sdma_$tag.log 2>&1 || { tail -30 gpurun_out/r2b_sdma_$tag.log; exit 1; }
  echo -n "$tag "; summ gpurun_out/r2b_sdma_$tag.log
}
b def1 VGATE_X=0
b nosdma1 HSA_ENABLE_SDMA=0
b def2 VGATE_X=0
b nosdma2 HSA_ENABLE_SDMA=0
rm -rf gpurun_out/prof_s
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_s -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/r2b_sdma_prof.log 2>&1 || { tail -30 gpurun_out/r2b_sdma_prof.log; exit 1; }
DB=$(find gpurun_out/prof_s -name "*results.db" | head -1)
python - "$DB" <<'PY' > gpurun_out/r2b_sdma_seq.log 2>&1 || true
import sqlite3, sys
con = sqlite3.connect(sys.argv[1])
tabs = [r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")]
print(tabs)
for t in tabs:
    if 'memory_copy' in t.lower() or 'kernel' in t.lower():
        cols = [r[1] for r in con.execute(f"pragma table_info('{t}')")]
        print(t, cols)
PY
cat gpurun_out/r2b_sdma_seq.log | head -30
rm -rf gpurun_out/prof_s_keep; mv gpurun_out/prof_s gpurun_out/prof_s_keep
