# Round 3 (session 2): wide int4 decode kernel — tests, in-engine AWQ sweep (qkv, o, gate_up incl. ntb -8)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "awq_wide" > gpurun_out/r3b_awqw1_tests.log 2>&1 || { tail -40 gpurun_out/r3b_awqw1_tests.log; exit 1; }
tail -1 gpurun_out/r3b_awqw1_tests.log
timeout -k 10 600 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --quantization awq --kinds gate_up,qkv,o > gpurun_out/r3b_awqw1_sweep.log 2>&1 || { tail -30 gpurun_out/r3b_awqw1_sweep.log; exit 1; }
grep '^{' gpurun_out/r3b_awqw1_sweep.log
