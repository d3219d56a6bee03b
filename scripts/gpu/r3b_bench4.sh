# Round 3 (session 2): driver bench with the engine idle / prefill-step accounting
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3b_bench4.log 2>&1 || { tail -30 gpurun_out/r3b_bench4.log; exit 1; }
tail -1 gpurun_out/r3b_bench4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','timed_engine_steps','timed_engine_idle_ms','timed_prefill_steps','max_cycle_tokens_seqs')})"
