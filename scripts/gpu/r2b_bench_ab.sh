# engine bench A/B: the tree's build vs ab/_C_base.so (bf16 headline, then AWQ + security)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
SO=vgate/_C.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/new.so
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','p50_s','p99_s','engine_avg_gpu_ms')})"; }
b() {
  tag=$1; shift
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 "$@" > gpurun_out/r2b_bab_$tag.log 2>&1 || { tail -30 gpurun_out/r2b_bab_$tag.log; exit 1; }
  echo -n "$tag "; summ gpurun_out/r2b_bab_$tag.log
}
b new_bf16
b new_awq --quantization awq --security
cp ab/_C_base.so $SO
b base_bf16
b base_awq --quantization awq --security
cp /tmp/new.so $SO
b new_bf16_2
b new_awq_2 --quantization awq --security
