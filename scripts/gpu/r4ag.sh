# Round 4: single-launch sampler block width A/B (256 / 512 / 1024 threads), probe + decode step, one box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for nt in 256 512 1024 256; do
  VGATE_SAMPLE_GRAN_THREADS=$nt timeout -k 10 300 python -u benchmarks/sampler_probe.py > gpurun_out/r4ag_probe_$nt.log 2>&1 || { tail -30 gpurun_out/r4ag_probe_$nt.log; exit 1; }
  echo "threads $nt"; grep '^{' gpurun_out/r4ag_probe_$nt.log | head -1 | cut -c280-600
done
for nt in 256 1024; do
  VGATE_SAMPLE_GRAN_THREADS=$nt timeout -k 10 300 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --baseline-only > gpurun_out/r4ag_step_$nt.log 2>&1 || { tail -20 gpurun_out/r4ag_step_$nt.log; exit 1; }
  echo "step threads $nt"; grep '^{' gpurun_out/r4ag_step_$nt.log
done
