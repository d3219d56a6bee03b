# Round 5: decode-GEMM-shaped streaming probe (layout / waves / activation loads / group depth)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out build
hipcc --offload-arch=gfx950 -O3 -o build/decode_stream_probe benchmarks/probes/decode_stream_probe.hip
timeout -k 10 240 ./build/decode_stream_probe > gpurun_out/r5e_stream.log 2>&1 || { tail -20 gpurun_out/r5e_stream.log; exit 1; }
cat gpurun_out/r5e_stream.log
