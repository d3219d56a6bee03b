# Round 5: int4 wide decode GEMM anatomy (gate_up shape)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out build
hipcc --offload-arch=gfx950 -O3 -I csrc/kernels -o build/awq_wide_anatomy benchmarks/probes/awq_wide_anatomy.hip
timeout -k 10 240 ./build/awq_wide_anatomy > gpurun_out/r5i_awq.log 2>&1 || { tail -20 gpurun_out/r5i_awq.log; exit 1; }
cat gpurun_out/r5i_awq.log
