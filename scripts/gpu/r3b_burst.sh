# Round 3 (session 2): the wave-arrival prefill step (8 prompts of 47 tokens, no decode rows): device time + kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/mixed_step.py --batch 1 --burst 8 --prompts 47 > gpurun_out/r3b_burst.log 2>&1 || { tail -30 gpurun_out/r3b_burst.log; exit 1; }
grep '^{"case' gpurun_out/r3b_burst.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b_burst_prof -o burst -- python3 -u benchmarks/mixed_step.py --batch 1 --burst 8 --prompts 47 --iters 20 > gpurun_out/r3b_burst_prof.log 2>&1 || { tail -30 gpurun_out/r3b_burst_prof.log; exit 1; }
