# Round 3 (session 2): HEAD evidence — GPU tier, smoke, driver bench x2, AWQ+security bench, rocprofv3 kernel trace of the driver bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r3b_head_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r3b_head_tests.log; exit 1; }
tail -1 gpurun_out/r3b_head_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3b_head_smoke.log 2>&1 || { tail -30 gpurun_out/r3b_head_smoke.log; exit 1; }
tail -1 gpurun_out/r3b_head_smoke.log | cut -c1-120
for i in 1 2; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3b_head_bench_$i.log 2>&1 || { tail -30 gpurun_out/r3b_head_bench_$i.log; exit 1; }
tail -1 gpurun_out/r3b_head_bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bf16', {k: d[k] for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','timed_engine_idle_ms','timed_prefill_steps','timed_eager_steps')})"
done
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r3b_head_awq.log 2>&1 || { tail -30 gpurun_out/r3b_head_awq.log; exit 1; }
tail -1 gpurun_out/r3b_head_awq.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('awq', {k: d[k] for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','timed_engine_idle_ms','timed_prefill_steps')})"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b_head_prof -o bench -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3b_head_prof.log 2>&1 || { tail -30 gpurun_out/r3b_head_prof.log; exit 1; }
tail -1 gpurun_out/r3b_head_prof.log | cut -c1-200
