set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2b_ring_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r2b_ring_tests.log; exit 1; }
tail -1 gpurun_out/r2b_ring_tests.log
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','p50_s','p99_s','engine_avg_gpu_ms','max_gpu_step_ms')})"; }
b() {
  tag=$1; shift
  timeout -k 10 300 env "$@" python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2b_ring_$tag.log 2>&1 || { tail -30 gpurun_out/r2b_ring_$tag.log; exit 1; }
  echo -n "$tag "; summ gpurun_out/r2b_ring_$tag.log
}
b ring1 VGATE_RING_IDS=1
b copy1 VGATE_RING_IDS=0
b ring2 VGATE_RING_IDS=1
b copy2 VGATE_RING_IDS=0
rm -rf gpurun_out/prof_r
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_r -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/r2b_ring_prof.log 2>&1 || { tail -30 gpurun_out/r2b_ring_prof.log; exit 1; }
DB=$(find gpurun_out/prof_r -name "*results.db" | head -1)
python benchmarks/step_boundary.py $DB --show 1 > gpurun_out/r2b_ring_boundary.log 2>&1 || true
cat gpurun_out/r2b_ring_boundary.log | cut -c1-200
rm -rf gpurun_out/prof_r
