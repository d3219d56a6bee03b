# Round 5: Qwen bf16 QKV projection on the tile-kernel wave counts inside the fused launch (A/B by plan entry)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # $1 = plan entry (python literal or none), rest = script + args
  local e=$1; shift
  python -u -c "import sys, runpy; import vgate.models.decode_plans as d; e = $e; e is not None and d.PLANS.__setitem__((2048, 1536, 'qkv', 'dense'), e); sys.argv = sys.argv[1:]; runpy.run_path(sys.argv[0], run_name='__main__')" "$@"
}
for e in None "(4,1,0)" "(6,1,0)" "(8,2,0)" None; do
timeout -k 10 300 bash -c "$(declare -f run); run \"$e\" benchmarks/timeline.py --batch 8 --ctx 100" > gpurun_out/r5ar_tl.log 2>&1 || { tail -30 gpurun_out/r5ar_tl.log; exit 1; }
echo "$e $(grep -o '"launches": [0-9]*, "step_us": [0-9.]*' gpurun_out/r5ar_tl.log | head -1) $(grep -o '"[a-z_]*qa[a-z_]*\[[0-9]*\]": {"n": 28, "avg_span_us": [0-9.]*' gpurun_out/r5ar_tl.log | head -1)"
done
