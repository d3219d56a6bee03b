# Round 4 HEAD check after the fused TP epilogue: decode-step timeline x2 + driver bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r4aa_tl1.log 2>&1 || { tail -30 gpurun_out/r4aa_tl1.log; exit 1; }
head -c 300 gpurun_out/r4aa_tl1.log; echo
timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only > gpurun_out/r4aa_step.log 2>&1 || { tail -30 gpurun_out/r4aa_step.log; exit 1; }
grep '^{' gpurun_out/r4aa_step.log | head -3
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4aa_bench.log 2>&1 || { tail -30 gpurun_out/r4aa_bench.log; exit 1; }
grep '^{' gpurun_out/r4aa_bench.log
