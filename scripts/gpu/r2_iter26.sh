set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/sampler_probe.py > gpurun_out/r2_sprobe26.log 2>&1 || { tail -30 gpurun_out/r2_sprobe26.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r2_sprobe26.log
