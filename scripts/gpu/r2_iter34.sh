set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "awq" --timeout 120 --timeout-method thread > gpurun_out/r2_awq34.log 2>&1 || { echo T_FAIL; tail -50 gpurun_out/r2_awq34.log; exit 1; }
tail -1 gpurun_out/r2_awq34.log
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_eng34.log 2>&1 || { echo E_FAIL; tail -50 gpurun_out/r2_eng34.log; exit 1; }
tail -1 gpurun_out/r2_eng34.log
for h in 1 0; do
VGATE_AWQ_NORM_HANDOFF=$h timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r2_bench34_awq_$h.json.log 2>&1 || { tail -20 gpurun_out/r2_bench34_awq_$h.json.log; exit 1; }
echo "handoff=$h $(tail -1 gpurun_out/r2_bench34_awq_$h.json.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','p50_s','p99_s','engine_avg_gpu_ms')})")"
done
