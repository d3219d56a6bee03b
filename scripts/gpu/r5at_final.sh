# Round 5 last check at HEAD: GPU tier (timed), smoke, driver bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5at_tier.log 2>&1 || { echo T_FAIL; tail -40 gpurun_out/r5at_tier.log; exit 1; }
echo "gpu tier wall s: $(( $(date +%s) - t0 ))" | tee -a gpurun_out/r5at_tier.log
tail -2 gpurun_out/r5at_tier.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5at_smoke.log 2>&1 || { tail -30 gpurun_out/r5at_smoke.log; exit 1; }
tail -1 gpurun_out/r5at_smoke.log | cut -c1-100
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5at_bench.log 2>&1 || { tail -30 gpurun_out/r5at_bench.log; exit 1; }
tail -1 gpurun_out/r5at_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','max_gpu_step_ms','timed_engine_idle_ms')})"
