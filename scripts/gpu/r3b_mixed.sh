# Round 3 (session 2): mixed-step (decode rows + one prompt) device time, bf16 and AWQ; kernel stats of the P=48 case
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/mixed_step.py > gpurun_out/r3b_mixed_bf16.log 2>&1 || { tail -30 gpurun_out/r3b_mixed_bf16.log; exit 1; }
grep '^{' gpurun_out/r3b_mixed_bf16.log
timeout -k 10 300 python -u benchmarks/mixed_step.py --quantization awq > gpurun_out/r3b_mixed_awq.log 2>&1 || { tail -30 gpurun_out/r3b_mixed_awq.log; exit 1; }
grep '^{' gpurun_out/r3b_mixed_awq.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b_mixed_prof -o mixed -- python3 -u benchmarks/mixed_step.py --prompts 48 --iters 20 > gpurun_out/r3b_mixed_prof.log 2>&1 || { tail -30 gpurun_out/r3b_mixed_prof.log; exit 1; }
find gpurun_out/r3b_mixed_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -40 {} | cut -d, -f1-8'
