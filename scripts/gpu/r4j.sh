# Round 4: stream-K decode GEMM variants vs the tile-per-block kernels, per projection (cold weights, in-graph)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_streamk_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4j_tests.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/r4j_tests.log; exit 1; }
tail -1 gpurun_out/r4j_tests.log
for m in qwen llama70b_tp8 llama8b; do
  timeout -k 10 300 python -u benchmarks/sk_probe.py --model $m > gpurun_out/r4j_probe_$m.log 2>&1 || { tail -30 gpurun_out/r4j_probe_$m.log; exit 1; }
  grep '^{' gpurun_out/r4j_probe_$m.log
done
