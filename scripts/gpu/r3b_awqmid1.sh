# Round 3 (session 2): int4 medium-M kernel — tests, AWQ engine correctness, AWQ mixed steps int4-mid vs dequant scratch
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "awq" > gpurun_out/r3b_awqmid1_tests.log 2>&1 || { tail -40 gpurun_out/r3b_awqmid1_tests.log; exit 1; }
tail -1 gpurun_out/r3b_awqmid1_tests.log
for v in 1 0; do
VGATE_AWQ_MID=$v timeout -k 10 300 python -u benchmarks/mixed_step.py --quantization awq --prompts 16,32,48 > gpurun_out/r3b_awqmid1_mixed_$v.log 2>&1 || { tail -30 gpurun_out/r3b_awqmid1_mixed_$v.log; exit 1; }
echo "VGATE_AWQ_MID=$v"; grep '^{"case' gpurun_out/r3b_awqmid1_mixed_$v.log
done
