# Parameterised GPU-box driver: every step runs under its own time limit, steps chain with
# `&&`-semantics (the script stops at the first failure), logs land in gpurun_out/<tag>_*.
#
#   gpurun -- bash scripts/gpu/run.sh <tag> <task> [<task> ...]
#
# tasks:
#   tier        GPU test tier (timed), tail of the log
#   smoke       __graft_entry__.smoke()
#   bench       driver bench (python bench.py --gpus 1 --steps 20 --warmup 5)
#   bench2      the driver bench twice (box-noise check)
#   awq         AWQ + security driver bench
#   timeline    graph-replayed decode step timeline (Qwen batch 8 / ctx 100)
#   ptimeline   prefill (448-row) step timeline
#   rocprof     rocprofv3 --kernel-trace --stats of the driver bench -> gpurun_out/<tag>_prof
#   py:<file>   python -u <file> (a benchmark / probe; extra args via PYARGS env)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
summ='import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print({k: d.get(k) for k in ("value","p50_s","p99_s","dtype","engine_avg_gpu_ms","engine_avg_step_ms","max_gpu_step_ms","timed_engine_idle_ms","timed_wall_ms_accounted")})'
fail() { echo "FAIL $1"; tail -40 "$2"; exit 1; }
for task in "$@"; do
  log=gpurun_out/${tag}_${task//[:\/.]/_}.log
  t0=$(date +%s)
  case $task in
    tier)
      timeout -k 10 420 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$log" 2>&1 || fail tier "$log"
      echo "gpu tier wall s: $(( $(date +%s) - t0 ))" | tee -a "$log"; tail -2 "$log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 || fail smoke "$log"
      tail -1 "$log" | cut -c1-160 ;;
    bench)
      timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$log" 2>&1 || fail bench "$log"
      tail -1 "$log" | python3 -c "$summ" ;;
    bench2)
      for i in 1 2; do
        timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "${log%.log}_$i.log" 2>&1 || fail bench2 "${log%.log}_$i.log"
        tail -1 "${log%.log}_$i.log" | python3 -c "$summ"
      done ;;
    awq)
      timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > "$log" 2>&1 || fail awq "$log"
      tail -1 "$log" | python3 -c "$summ" ;;
    timeline)
      timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 ${PYARGS:-} > "$log" 2>&1 || fail timeline "$log"
      grep -m1 -o '"launches": [0-9]*, "step_us": [0-9.]*' "$log" ;;
    ptimeline)
      timeout -k 10 300 python -u benchmarks/timeline.py --prefill --batch 8 --ctx 50 ${PYARGS:-} > "$log" 2>&1 || fail ptimeline "$log"
      grep -m1 -o '"launches": [0-9]*, "step_us": [0-9.]*' "$log" ;;
    rocprof)
      timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$log" 2>&1 || fail rocprof "$log"
      tail -1 "$log" | python3 -c "$summ" ;;
    py:*)
      timeout -k 10 400 python -u "${task#py:}" ${PYARGS:-} > "$log" 2>&1 || fail "$task" "$log"
      grep '^{' "$log" | tail -20 ;;
    *) echo "unknown task $task"; exit 2 ;;
  esac
done
