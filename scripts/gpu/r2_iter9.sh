set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/micro_gpu.py --only attn > gpurun_out/r2_attn9.log 2>&1 || { tail -20 gpurun_out/r2_attn9.log; exit 1; }
grep attention gpurun_out/r2_attn9.log
timeout -k 10 300 python -u benchmarks/decode_sweep.py --kinds gate_up,lm_head > gpurun_out/r2_sweep9.log 2>&1 || { tail -20 gpurun_out/r2_sweep9.log; exit 1; }
grep '^{' gpurun_out/r2_sweep9.log | tail -16
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench9.json.log 2>&1 || { tail -20 gpurun_out/r2_bench9.json.log; exit 1; }
tail -1 gpurun_out/r2_bench9.json.log
