# Round 5 baseline at HEAD: GPU tier, smoke, driver bench, rocprof kernel table of the driver command
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r5a_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5a_tests.log; exit 1; }
echo "gpu tier wall s: $(( $(date +%s) - t0 ))" | tee -a gpurun_out/r5a_tests.log
tail -2 gpurun_out/r5a_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5a_smoke.log 2>&1 || { tail -30 gpurun_out/r5a_smoke.log; exit 1; }
tail -1 gpurun_out/r5a_smoke.log | cut -c1-200
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5a_bench.log 2>&1 || { tail -30 gpurun_out/r5a_bench.log; exit 1; }
tail -1 gpurun_out/r5a_bench.log | cut -c1-600
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/r5a_prof -o bench -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5a_prof_bench.log 2>&1 || { tail -30 gpurun_out/r5a_prof_bench.log; exit 1; }
python3 benchmarks/prof_summary.py /tmp/r5a_prof/bench_results.db --top 40 > gpurun_out/r5a_prof_kernels.txt
head -30 gpurun_out/r5a_prof_kernels.txt | cut -c1-150
