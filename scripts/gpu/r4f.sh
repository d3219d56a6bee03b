# Round 4: fused MLP fine phase stamps; decode timeline (1 replay vs back-to-back replays: the post-embedding hole); driver bench baseline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_mlp_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4f_mlp_test.log 2>&1 || { echo MLP_TEST_FAIL; tail -60 gpurun_out/r4f_mlp_test.log; exit 1; }
tail -1 gpurun_out/r4f_mlp_test.log
timeout -k 10 240 python -u benchmarks/mlp_probe.py --b-early 0 > gpurun_out/r4f_mlp_probe.log 2>&1 || { tail -30 gpurun_out/r4f_mlp_probe.log; exit 1; }
grep '^{' gpurun_out/r4f_mlp_probe.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 --replays 3 > gpurun_out/r4f_timeline.log 2>&1 || { tail -30 gpurun_out/r4f_timeline.log; exit 1; }
grep '"launches"' gpurun_out/r4f_timeline.log | cut -c1-400
grep '"kernel": "embedding"' gpurun_out/r4f_timeline.log | cut -c1-300
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4f_bench.log 2>&1 || { tail -30 gpurun_out/r4f_bench.log; exit 1; }
tail -1 gpurun_out/r4f_bench.log | cut -c1-900
