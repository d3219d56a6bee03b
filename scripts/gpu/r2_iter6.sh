set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -o /tmp/grid_barrier_probe benchmarks/grid_barrier_probe.hip
timeout -k 10 120 /tmp/grid_barrier_probe > gpurun_out/r2_grid_barrier.log 2>&1 || { echo PROBE_FAIL; cat gpurun_out/r2_grid_barrier.log; exit 1; }
cat gpurun_out/r2_grid_barrier.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_head -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_head_bench_prof.log 2>&1 || { tail -20 gpurun_out/r2_head_bench_prof.log; exit 1; }
grep '^{' gpurun_out/r2_head_bench_prof.log | tail -1
DB=$(ls /tmp/prof_head/*.db /tmp/prof_head/*/*.db 2>/dev/null | head -1)
echo "db=$DB"
python benchmarks/prof_summary.py "$DB" --top 45 > gpurun_out/r2_head_kernels.txt 2>&1 || true
head -50 gpurun_out/r2_head_kernels.txt
find /tmp/prof_head -name '*stats*.csv' -exec cp {} gpurun_out/ \; || true
ls /tmp/prof_head /tmp/prof_head/* | head
