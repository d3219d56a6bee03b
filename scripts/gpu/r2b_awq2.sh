set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "awq or sample" --timeout 120 --timeout-method thread > gpurun_out/r2b_awq2_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r2b_awq2_tests.log; exit 1; }
tail -1 gpurun_out/r2b_awq2_tests.log
AWQ_SWEEP_SHAPES=qkv,o_proj AWQ_SWEEP_CFGS="0:0:0,4:0:-2,4:0:1,2:0:1,8:0:1" timeout -k 10 300 python -u benchmarks/awq_sweep.py > gpurun_out/r2b_awq2_sweep.log 2>&1 || { tail -30 gpurun_out/r2b_awq2_sweep.log; exit 1; }
python - <<'PY'
import json
for line in open("gpurun_out/r2b_awq2_sweep.log"):
    if not line.startswith("{"): continue
    d = json.loads(line)
    print(d["shape"], [(r["waves"], r["splitk"], r["ntb"], r["span_us"], r["wall_us"]) for r in d["rows"]])
PY
timeout -k 10 300 python -u benchmarks/sampler_probe.py > gpurun_out/r2b_awq2_sprobe.log 2>&1 || { tail -30 gpurun_out/r2b_awq2_sprobe.log; exit 1; }
grep "sampler_us\|round_launches" gpurun_out/r2b_awq2_sprobe.log | cut -c1-300
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','p50_s','p99_s')})"; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2b_awq2_bf16_$i.log 2>&1 || { tail -30 gpurun_out/r2b_awq2_bf16_$i.log; exit 1; }
  echo -n "bf16_$i "; summ gpurun_out/r2b_awq2_bf16_$i.log
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r2b_awq2_awq_$i.log 2>&1 || { tail -30 gpurun_out/r2b_awq2_awq_$i.log; exit 1; }
  echo -n "awq_$i "; summ gpurun_out/r2b_awq2_awq_$i.log
done
