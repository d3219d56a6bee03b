# Round 5: decode GEMM anatomy (production kernel vs copies with one piece changed) + sampler launch time by mode
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out build
hipcc --offload-arch=gfx950 -O3 -I csrc/kernels -o build/decode_gemm_anatomy benchmarks/probes/decode_gemm_anatomy.hip
timeout -k 10 240 ./build/decode_gemm_anatomy > gpurun_out/r5f_anatomy.log 2>&1 || { tail -20 gpurun_out/r5f_anatomy.log; exit 1; }
cat gpurun_out/r5f_anatomy.log
timeout -k 10 240 python -u benchmarks/sampler_modes.py > gpurun_out/r5f_sampler.log 2>&1 || { tail -20 gpurun_out/r5f_sampler.log; exit 1; }
cat gpurun_out/r5f_sampler.log
