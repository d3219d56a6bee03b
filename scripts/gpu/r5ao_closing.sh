# Round 5 closing check at HEAD: smoke, driver bench x2, AWQ + security bench, decode timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5ao_smoke.log 2>&1 || { tail -30 gpurun_out/r5ao_smoke.log; exit 1; }
tail -1 gpurun_out/r5ao_smoke.log | cut -c1-120
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r5ao_tl.log 2>&1 || { tail -30 gpurun_out/r5ao_tl.log; exit 1; }
grep -o '"launches": [0-9]*, "step_us": [0-9.]*' gpurun_out/r5ao_tl.log | head -1
for i in 1 2; do
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5ao_bench_$i.log 2>&1 || { tail -30 gpurun_out/r5ao_bench_$i.log; exit 1; }
tail -1 gpurun_out/r5ao_bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','max_gpu_step_ms','timed_engine_idle_ms')})"
done
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r5ao_bench_awq.log 2>&1 || { tail -30 gpurun_out/r5ao_bench_awq.log; exit 1; }
tail -1 gpurun_out/r5ao_bench_awq.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','dtype')})"
