# Round 4 final HEAD evidence (1/2): GPU tier (timed), smoke, driver bench x2, rocprofv3 kernel trace of the driver command
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4f1_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r4f1_tests.log; exit 1; }
echo "gpu tier wall s: $(( $(date +%s) - t0 ))" | tee -a gpurun_out/r4f1_tests.log
tail -2 gpurun_out/r4f1_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f1_smoke.log 2>&1 || { tail -30 gpurun_out/r4f1_smoke.log; exit 1; }
tail -1 gpurun_out/r4f1_smoke.log | cut -c1-200
for i in 1 2; do
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4f1_bench_$i.log 2>&1 || { tail -30 gpurun_out/r4f1_bench_$i.log; exit 1; }
tail -1 gpurun_out/r4f1_bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','max_gpu_step_ms','max_gpu_step_bucket','timed_prefill_steps')})"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r4f1_prof -o bench -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4f1_prof_bench.log 2>&1 || { tail -30 gpurun_out/r4f1_prof_bench.log; exit 1; }
tail -1 gpurun_out/r4f1_prof_bench.log | cut -c1-200
python3 benchmarks/prof_summary.py /tmp/r4f1_prof/bench_results.db --top 45 > gpurun_out/r4f1_prof_kernels.txt
head -20 gpurun_out/r4f1_prof_kernels.txt | cut -c1-150
