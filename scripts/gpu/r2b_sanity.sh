set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r2b_sanity_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r2b_sanity_tests.log; exit 1; }
tail -1 gpurun_out/r2b_sanity_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2b_sanity_smoke.log 2>&1 || { tail -30 gpurun_out/r2b_sanity_smoke.log; exit 1; }
tail -1 gpurun_out/r2b_sanity_smoke.log | cut -c1-120
timeout -k 10 300 python -u bench.py > gpurun_out/r2b_sanity_bench_default.log 2>&1 || { tail -30 gpurun_out/r2b_sanity_bench_default.log; exit 1; }
tail -1 gpurun_out/r2b_sanity_bench_default.log | cut -c1-300
