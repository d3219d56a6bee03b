# Round 5: MALL / HBM streaming probe (cold vs MALL-warm vs L2-warm) + the decode-step timeline (gaps per kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out build
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -o build/mall_stream_probe benchmarks/probes/mall_stream_probe.hip
timeout -k 10 240 ./build/mall_stream_probe > gpurun_out/r5d_mall.log 2>&1 || { tail -20 gpurun_out/r5d_mall.log; exit 1; }
cat gpurun_out/r5d_mall.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r5d_timeline.log 2>&1 || { tail -30 gpurun_out/r5d_timeline.log; exit 1; }
tail -3 gpurun_out/r5d_timeline.log | cut -c1-3000
# load generator in its own process (as the reference's bench_load.py) vs in the server process
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --client-process > gpurun_out/r5d_bench_cproc.log 2>&1 || { tail -30 gpurun_out/r5d_bench_cproc.log; exit 1; }
tail -1 gpurun_out/r5d_bench_cproc.log | cut -c1-1200
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5d_bench_inproc.log 2>&1 || { tail -30 gpurun_out/r5d_bench_inproc.log; exit 1; }
tail -1 gpurun_out/r5d_bench_inproc.log | cut -c1-1200
