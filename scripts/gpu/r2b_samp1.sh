set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "sample" --timeout 120 --timeout-method thread > gpurun_out/r2b_samp_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r2b_samp_tests.log; exit 1; }
tail -1 gpurun_out/r2b_samp_tests.log
timeout -k 10 300 python -u benchmarks/sampler_probe.py > gpurun_out/r2b_samp_probe.log 2>&1 || { tail -30 gpurun_out/r2b_samp_probe.log; exit 1; }
grep "^{" gpurun_out/r2b_samp_probe.log | cut -c1-400
