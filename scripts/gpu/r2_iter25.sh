set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 0 1 0; do
VGATE_LM_SAMPLE_PARTS=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2_bench25_$v.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/r2_bench25_$v.log; exit 1; }
echo "lm_parts=$v $(tail -1 gpurun_out/r2_bench25_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','p50_s','p99_s','engine_avg_gpu_ms')})")"
done
VGATE_LM_SAMPLE_PARTS=1 timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r2_tl25.log 2>&1 || { tail -30 gpurun_out/r2_tl25.log; exit 1; }
head -2 gpurun_out/r2_tl25.log | cut -c1-2500
