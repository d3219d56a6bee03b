# Round 3 (session 2): load client in-process vs separate process (engine idle per wave boundary)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for mode in "" "--client-process" "" "--client-process"; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 $mode > gpurun_out/r3b_bench5.log 2>&1 || { tail -30 gpurun_out/r3b_bench5.log; exit 1; }
tail -1 gpurun_out/r3b_bench5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode', {k: d[k] for k in ('value','p50_s','p99_s','timed_engine_idle_ms','timed_prefill_steps')})"
done
