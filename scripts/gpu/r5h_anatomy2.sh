# Round 5: decode GEMM anatomy with the activation-preload variant and the NORM 3 (hand-off) consumer
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out build
hipcc --offload-arch=gfx950 -O3 -I csrc/kernels -o build/decode_gemm_anatomy benchmarks/probes/decode_gemm_anatomy.hip
timeout -k 10 240 ./build/decode_gemm_anatomy > gpurun_out/r5h_anatomy.log 2>&1 || { tail -20 gpurun_out/r5h_anatomy.log; exit 1; }
cat gpurun_out/r5h_anatomy.log
