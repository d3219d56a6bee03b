# Round 4: rocprofv3 kernel table of the AWQ + security driver command (BASELINE config 5)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/r4an_prof -o bench -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --quantization awq --security > gpurun_out/r4an_prof_bench.log 2>&1 || { tail -30 gpurun_out/r4an_prof_bench.log; exit 1; }
grep '^{' gpurun_out/r4an_prof_bench.log | tail -1 | cut -c1-300
python3 benchmarks/prof_summary.py /tmp/r4an_prof/bench_results.db --top 40 > gpurun_out/r4an_prof_kernels.txt
head -24 gpurun_out/r4an_prof_kernels.txt | cut -c1-150
