set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp


bash scripts/gpu/run.sh r6k tier smoke timeline bench || exit 1
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r6k_awq_w3.log 2>&1 || { tail -30 gpurun_out/r6k_awq_w3.log; exit 1; }
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security --idle-window-ms 0 > gpurun_out/r6k_awq_w0.log 2>&1 || { tail -30 gpurun_out/r6k_awq_w0.log; exit 1; }
for f in w3 w0; do tail -1 gpurun_out/r6k_awq_$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', {k: d.get(k) for k in ('value','p50_s','p99_s','timed_prefill_steps','timed_waves','wave_breakdown_ms','timed_engine_idle_ms','timed_engine_coalesce_ms','timed_wall_ms','timed_wall_ms_accounted')})"; done
timeout -k 10 300 python -u benchmarks/ttft_probe.py --model meta-llama/Meta-Llama-3-8B-Instruct --lens 512 2048 4096 > gpurun_out/r6k_ttft.log 2>&1 || { tail -30 gpurun_out/r6k_ttft.log; exit 1; }
grep '^{' gpurun_out/r6k_ttft.log | tail -3
