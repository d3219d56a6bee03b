# Round 4: fused MLP probe: x waited for before the weight burst (default) vs not; down weights late vs early
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_mlp_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4e_mlp_test.log 2>&1 || { echo MLP_TEST_FAIL; tail -60 gpurun_out/r4e_mlp_test.log; exit 1; }
tail -1 gpurun_out/r4e_mlp_test.log
for be in 0 1 2; do
timeout -k 10 240 python -u benchmarks/mlp_probe.py --b-early $be > gpurun_out/r4e_mlp_probe_$be.log 2>&1 || { tail -30 gpurun_out/r4e_mlp_probe_$be.log; exit 1; }
echo "b_early=$be"; grep '^{' gpurun_out/r4e_mlp_probe_$be.log
done
