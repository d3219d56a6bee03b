# Round 3 (session 2): per-kernel times of the P=48 mixed step (bucket [64, 8]) with the tuned medium plans and with the wide gate_up kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in tuned wide; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b_mid3_$m -o mixed -- python3 -u benchmarks/mixed_step.py --medium $m --prompts 48 --iters 20 > gpurun_out/r3b_mid3_$m.log 2>&1 || { tail -30 gpurun_out/r3b_mid3_$m.log; exit 1; }
grep '^{"case' gpurun_out/r3b_mid3_$m.log
done
