# Round 5: prefill-step timeline (8 x 50-token prompts -> 448-token bucket) and decode-attention phases
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/timeline.py --prefill --batch 8 --ctx 50 > gpurun_out/r5q_prefill_timeline.log 2>&1 || { tail -30 gpurun_out/r5q_prefill_timeline.log; exit 1; }
grep -h '"step_us"' gpurun_out/r5q_prefill_timeline.log | cut -c1-120
timeout -k 10 200 python -u benchmarks/attn_phases.py > gpurun_out/r5q_attn_phases.log 2>&1 || { tail -30 gpurun_out/r5q_attn_phases.log; exit 1; }
cat gpurun_out/r5q_attn_phases.log | cut -c1-300
