# Round 4: driver bench at HEAD (ring prefill tiles + finer prefill buckets + DPP sampler reductions), twice, and a prefill-step timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4m_bench_$i.log 2>&1 || { tail -30 gpurun_out/r4m_bench_$i.log; exit 1; }
tail -1 gpurun_out/r4m_bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','max_gpu_step_ms','max_gpu_step_bucket','boot_s','timed_prefill_steps')})"
done
timeout -k 10 300 python -u benchmarks/mixed_step.py --help > /dev/null 2>&1; true
