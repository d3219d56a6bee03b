# Round 3 (session 2): int4 medium kernel at decode M (hand-off modes) — tests, in-engine AWQ sweep of qkv / o / down
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "awq_mid" > gpurun_out/r3b_awqmid2_tests.log 2>&1 || { tail -40 gpurun_out/r3b_awqmid2_tests.log; exit 1; }
tail -1 gpurun_out/r3b_awqmid2_tests.log
timeout -k 10 600 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --quantization awq --kinds qkv,o,down > gpurun_out/r3b_awqmid2_sweep.log 2>&1 || { tail -30 gpurun_out/r3b_awqmid2_sweep.log; exit 1; }
grep '^{' gpurun_out/r3b_awqmid2_sweep.log
