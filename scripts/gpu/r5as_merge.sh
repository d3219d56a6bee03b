# Round 5: decode-attention merge over the waves that had chunks: tests, phases, decode timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or decode or engine or graph or flash" > gpurun_out/r5as.log 2>&1 || { tail -40 gpurun_out/r5as.log; exit 1; }
tail -1 gpurun_out/r5as.log
timeout -k 10 200 python -u benchmarks/qa_phases.py > gpurun_out/r5as_ph.log 2>&1 || { tail -30 gpurun_out/r5as_ph.log; exit 1; }
grep '^{' gpurun_out/r5as_ph.log
for i in 1 2; do
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r5as_tl.log 2>&1 || { tail -30 gpurun_out/r5as_tl.log; exit 1; }
echo "$(grep -o '"launches": [0-9]*, "step_us": [0-9.]*' gpurun_out/r5as_tl.log | head -1) $(grep -o '"qkv_attn\[192\]": {"n": 28, "avg_span_us": [0-9.]*' gpurun_out/r5as_tl.log | head -1)"
done
