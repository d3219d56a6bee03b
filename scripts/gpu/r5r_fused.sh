# Round 5: fused producer/consumer launch probe (latency-bound producer + weight-streaming consumer in one launch)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out build
hipcc --offload-arch=gfx950 -O3 -o build/fused_pair_probe benchmarks/probes/fused_pair_probe.hip
timeout -k 10 60 ./build/fused_pair_probe > gpurun_out/r5r_fused.log 2>&1 || { tail -20 gpurun_out/r5r_fused.log; exit 1; }
cat gpurun_out/r5r_fused.log
