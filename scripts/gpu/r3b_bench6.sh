# Round 3 (session 2): idle admission window (coalesce a wave's arrivals into one prefill step) A/B, both client modes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "3.0 0.6 " "0 0 " "3.0 0.6 --client-process" "0 0 --client-process" "3.0 0.6 " "0 0 "; do
set -- $cfg
VGATE_IDLE_BATCH_WINDOW_MS=$1 VGATE_IDLE_BATCH_GAP_MS=$2 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 $3 > gpurun_out/r3b_bench6.log 2>&1 || { tail -30 gpurun_out/r3b_bench6.log; exit 1; }
tail -1 gpurun_out/r3b_bench6.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', {k: d[k] for k in ('value','p50_s','p99_s','timed_engine_idle_ms','timed_prefill_steps')})"
done
