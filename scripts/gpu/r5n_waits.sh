# Round 5: decode GEMM load/wait structure (unconditional activation / epilogue loads, hoist pins, loop peel),
# int4 kernel deletions: GPU tier, bf16 + AWQ timelines, bf16 + AWQ benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r5n_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5n_tests.log; exit 1; }
tail -2 gpurun_out/r5n_tests.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r5n_timeline_bf16.log 2>&1 || { tail -30 gpurun_out/r5n_timeline_bf16.log; exit 1; }
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 --quantization awq > gpurun_out/r5n_timeline_awq.log 2>&1 || { tail -30 gpurun_out/r5n_timeline_awq.log; exit 1; }
grep -h '"step_us"' gpurun_out/r5n_timeline_bf16.log gpurun_out/r5n_timeline_awq.log | cut -c1-100
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5n_bench.log 2>&1 || { tail -30 gpurun_out/r5n_bench.log; exit 1; }
tail -1 gpurun_out/r5n_bench.log | cut -c1-300
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r5n_bench_awq.log 2>&1 || { tail -30 gpurun_out/r5n_bench_awq.log; exit 1; }
tail -1 gpurun_out/r5n_bench_awq.log | cut -c1-300
