# Round 4: sampler probe on engine logits with the single-launch sampler (greedy / temperature / top-p, nseg caps)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/sampler_probe.py > gpurun_out/r4ae_probe.log 2>&1 || { tail -30 gpurun_out/r4ae_probe.log; exit 1; }
grep '^{' gpurun_out/r4ae_probe.log | cut -c1-600
VGATE_SAMPLE_SINGLE=0 timeout -k 10 300 python -u benchmarks/sampler_probe.py > gpurun_out/r4ae_probe_pass.log 2>&1 || { tail -30 gpurun_out/r4ae_probe_pass.log; exit 1; }
grep '^{' gpurun_out/r4ae_probe_pass.log | head -3 | cut -c1-600
