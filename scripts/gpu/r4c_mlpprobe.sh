# Round 4: fused MLP standalone probe (28 cold layers, phase stamps)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_mlp_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c_mlp_test.log 2>&1 || { echo MLP_TEST_FAIL; tail -60 gpurun_out/r4c_mlp_test.log; exit 1; }
tail -1 gpurun_out/r4c_mlp_test.log
timeout -k 10 240 python -u benchmarks/mlp_probe.py > gpurun_out/r4c_mlp_probe.log 2>&1 || { tail -30 gpurun_out/r4c_mlp_probe.log; exit 1; }
cat gpurun_out/r4c_mlp_probe.log | grep '^{'
