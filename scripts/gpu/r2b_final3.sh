# HEAD evidence: GPU tier, two driver-command bench runs, rocprofv3 kernel trace of the driver command,
# launch timeline of a decode step, AWQ bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r2b_final3_gpu_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r2b_final3_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r2b_final3_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2b_final3_smoke.log 2>&1 || { tail -30 gpurun_out/r2b_final3_smoke.log; exit 1; }
tail -1 gpurun_out/r2b_final3_smoke.log | cut -c1-200
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2b_final3_bench$i.log 2>&1 || { tail -30 gpurun_out/r2b_final3_bench$i.log; exit 1; }
  tail -1 gpurun_out/r2b_final3_bench$i.log | cut -c1-400
done
rm -rf /tmp/prof_final3
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof_final3 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2b_final3_prof_bench.log 2>&1 || { tail -30 gpurun_out/r2b_final3_prof_bench.log; exit 1; }
DB=$(find /tmp/prof_final3 -name "*results.db" | head -1)
python benchmarks/prof_summary.py $DB --top 30 > gpurun_out/r2b_final3_kernels.txt 2>&1 || true
head -24 gpurun_out/r2b_final3_kernels.txt | cut -c1-160
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r2b_final3_timeline.log 2>&1 || { tail -30 gpurun_out/r2b_final3_timeline.log; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r2b_final3_awq.log 2>&1 || { tail -30 gpurun_out/r2b_final3_awq.log; exit 1; }
tail -1 gpurun_out/r2b_final3_awq.log | cut -c1-300
