set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "sample" --timeout 120 --timeout-method thread > gpurun_out/r2_s27.log 2>&1 || { echo S_FAIL; tail -60 gpurun_out/r2_s27.log; exit 1; }
tail -2 gpurun_out/r2_s27.log
timeout -k 10 300 python -u benchmarks/sampler_probe.py > gpurun_out/r2_sprobe27.log 2>&1 || { tail -30 gpurun_out/r2_sprobe27.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r2_sprobe27.log
