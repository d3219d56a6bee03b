# Round 3 (session 3): sampler launches — rejection rounds as launches (VGATE_SAMPLE_ROUND_LAUNCHES 1, default) vs 0 (pass 0 + the in-launch resume kernel only)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 1 0; do
VGATE_SAMPLE_ROUND_LAUNCHES=$n timeout -k 10 300 python -u benchmarks/sampler_probe.py > gpurun_out/r3c_sampler_$n.log 2>&1 || { tail -30 gpurun_out/r3c_sampler_$n.log; exit 1; }
echo "ROUND_LAUNCHES=$n"; grep '^{' gpurun_out/r3c_sampler_$n.log | cut -c1-220
done
