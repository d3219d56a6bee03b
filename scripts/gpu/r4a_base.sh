# Round 4: baseline on this round's boxes — decode-step timeline (Qwen2.5-1.5B, batch 8, ctx 100), sampler round-launch A/B, driver bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r4a_timeline.log 2>&1 || { tail -30 gpurun_out/r4a_timeline.log; exit 1; }
grep '"launches"' gpurun_out/r4a_timeline.log | cut -c1-300
for n in 1 0; do
VGATE_SAMPLE_ROUND_LAUNCHES=$n timeout -k 10 300 python -u benchmarks/sampler_probe.py > gpurun_out/r4a_sampler_$n.log 2>&1 || { tail -30 gpurun_out/r4a_sampler_$n.log; exit 1; }
echo "ROUND_LAUNCHES=$n"; grep '^{' gpurun_out/r4a_sampler_$n.log | cut -c1-220
done
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4a_bench.log 2>&1 || { tail -30 gpurun_out/r4a_bench.log; exit 1; }
tail -1 gpurun_out/r4a_bench.log | cut -c1-600
