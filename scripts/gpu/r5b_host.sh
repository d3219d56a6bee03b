# Round 5: GPU tier + smoke, then the driver bench with the lean server/client vs uvicorn/aiohttp (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r5b_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5b_tests.log; exit 1; }
echo "gpu tier wall s: $(( $(date +%s) - t0 ))" | tee -a gpurun_out/r5b_tests.log
tail -2 gpurun_out/r5b_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5b_smoke.log 2>&1 || { tail -30 gpurun_out/r5b_smoke.log; exit 1; }
tail -1 gpurun_out/r5b_smoke.log | cut -c1-200
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5b_bench.log 2>&1 || { tail -30 gpurun_out/r5b_bench.log; exit 1; }
tail -1 gpurun_out/r5b_bench.log | cut -c1-900
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --server uvicorn --client aiohttp > gpurun_out/r5b_bench_old.log 2>&1 || { tail -30 gpurun_out/r5b_bench_old.log; exit 1; }
tail -1 gpurun_out/r5b_bench_old.log | cut -c1-900
