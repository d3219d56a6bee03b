set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','p50_s','p99_s')})"; }
for t in a:2 b:1 c:2 d:1 e:3; do
  tag=${t%%:*}; v=${t##*:}
  timeout -k 10 300 env VGATE_SAMPLE_ROUND_LAUNCHES=$v python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2b_rl_$tag.log 2>&1 || { tail -30 gpurun_out/r2b_rl_$tag.log; exit 1; }
  echo -n "rounds=$v "; summ gpurun_out/r2b_rl_$tag.log
done
