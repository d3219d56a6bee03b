# Round 5: fused QKV + attention on tile / kx / int4 kernels: tests, engine parity, phases, timelines, benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "qkv_attention_fused or attention or decode" > gpurun_out/r5aa_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5aa_tests.log; exit 1; }
tail -1 gpurun_out/r5aa_tests.log
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5aa_engine.log 2>&1 || { echo E_FAIL; tail -60 gpurun_out/r5aa_engine.log; exit 1; }
tail -1 gpurun_out/r5aa_engine.log
timeout -k 10 200 python -u benchmarks/qa_phases.py --ctx 512 > gpurun_out/r5aa_phases.log 2>&1 || { tail -30 gpurun_out/r5aa_phases.log; exit 1; }
cat gpurun_out/r5aa_phases.log | grep '^{'
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 --quantization awq > gpurun_out/r5aa_timeline_awq.log 2>&1 || { tail -30 gpurun_out/r5aa_timeline_awq.log; exit 1; }
head -c 400 gpurun_out/r5aa_timeline_awq.log | tail -c 300; echo
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5aa_bench.log 2>&1 || { tail -30 gpurun_out/r5aa_bench.log; exit 1; }
tail -1 gpurun_out/r5aa_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','max_gpu_step_ms','timed_engine_idle_ms')})"
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r5aa_bench_awq.log 2>&1 || { tail -30 gpurun_out/r5aa_bench_awq.log; exit 1; }
tail -1 gpurun_out/r5aa_bench_awq.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','max_gpu_step_ms','dtype')})"
