# Round 3 (session 3): HEAD — AWQ + security bench, and a rocprofv3 kernel trace of the driver bench command summarised on the box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r3c_head_awq.log 2>&1 || { tail -30 gpurun_out/r3c_head_awq.log; exit 1; }
tail -1 gpurun_out/r3c_head_awq.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('awq', {k: d[k] for k in ('value','p50_s','p99_s','timed_engine_idle_ms','timed_prefill_steps')})"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r3c_headprof -o bench -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3c_headprof_bench.log 2>&1 || { tail -30 gpurun_out/r3c_headprof_bench.log; exit 1; }
tail -1 gpurun_out/r3c_headprof_bench.log | cut -c1-200
python3 benchmarks/prof_summary.py /tmp/r3c_headprof/bench_results.db --top 45 > gpurun_out/r3c_headprof_kernels.txt
head -14 gpurun_out/r3c_headprof_kernels.txt | cut -c1-150
