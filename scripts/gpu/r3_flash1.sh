# Round 3: flash prefill attention (tests + throughput), then the block-rotation A/B (scripts/gpu/r3_rot1.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "prefill or attention" > gpurun_out/r3_flash1_tests.log 2>&1 || { tail -40 gpurun_out/r3_flash1_tests.log; exit 1; }
tail -2 gpurun_out/r3_flash1_tests.log
timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py > gpurun_out/r3_flash1_bench.log 2>&1 || { tail -30 gpurun_out/r3_flash1_bench.log; exit 1; }
grep '{' gpurun_out/r3_flash1_bench.log
bash scripts/gpu/r3_rot1.sh
