# Round 3 (session 2): driver bench (bf16) x2 and AWQ + security x2 at HEAD (medium-M plans, int4 medium kernel, AWQ decode plans)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3b_bench3_$i.log 2>&1 || { tail -30 gpurun_out/r3b_bench3_$i.log; exit 1; }
tail -1 gpurun_out/r3b_bench3_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bf16', d['value'], d['p50_s'], d['p99_s'], d['engine_avg_gpu_ms'])"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r3b_bench3_awq_$i.log 2>&1 || { tail -30 gpurun_out/r3b_bench3_awq_$i.log; exit 1; }
tail -1 gpurun_out/r3b_bench3_awq_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('awq', d['value'], d['p50_s'], d['p99_s'], d['engine_avg_gpu_ms'])"
done
