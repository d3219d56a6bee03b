# Round 5 HEAD evidence (fused QKV + attention, wide prefill tiles): GPU tier (timed), smoke, driver bench x2, rocprofv3 kernel tables of the bf16 driver
# command and of the AWQ + security command, AWQ bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5h_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5h_tests.log; exit 1; }
echo "gpu tier wall s: $(( $(date +%s) - t0 ))" | tee -a gpurun_out/r5h_tests.log
tail -2 gpurun_out/r5h_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5h_smoke.log 2>&1 || { tail -30 gpurun_out/r5h_smoke.log; exit 1; }
tail -1 gpurun_out/r5h_smoke.log | cut -c1-200
for i in 1 2; do
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5h_bench_$i.log 2>&1 || { tail -30 gpurun_out/r5h_bench_$i.log; exit 1; }
tail -1 gpurun_out/r5h_bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','max_gpu_step_ms','max_gpu_step_bucket','timed_engine_idle_ms')})"
done
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r5h_bench_awq.log 2>&1 || { tail -30 gpurun_out/r5h_bench_awq.log; exit 1; }
tail -1 gpurun_out/r5h_bench_awq.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','max_gpu_step_ms','dtype')})"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r5h_prof -o bench -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5h_prof_bench.log 2>&1 || { tail -30 gpurun_out/r5h_prof_bench.log; exit 1; }
tail -1 gpurun_out/r5h_prof_bench.log | cut -c1-200
python3 benchmarks/prof_summary.py /tmp/r5h_prof/bench_results.db --top 45 > gpurun_out/r5h_prof_kernels.txt
head -20 gpurun_out/r5h_prof_kernels.txt | cut -c1-150
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/r5h_aprof -o bench -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r5h_aprof_bench.log 2>&1 || { tail -30 gpurun_out/r5h_aprof_bench.log; exit 1; }
python3 benchmarks/prof_summary.py /tmp/r5h_aprof/bench_results.db --top 40 > gpurun_out/r5h_aprof_kernels.txt
head -16 gpurun_out/r5h_aprof_kernels.txt | cut -c1-150
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r5h_tl_decode.log 2>&1 || { tail -30 gpurun_out/r5h_tl_decode.log; exit 1; }
timeout -k 10 300 python -u benchmarks/timeline.py --prefill --batch 8 --ctx 50 > gpurun_out/r5h_tl_prefill.log 2>&1 || { tail -30 gpurun_out/r5h_tl_prefill.log; exit 1; }
grep -o '"launches": [0-9]*, "step_us": [0-9.]*' gpurun_out/r5h_tl_decode.log gpurun_out/r5h_tl_prefill.log | head -2
