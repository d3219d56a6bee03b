# ad-hoc GPU batch (the current experiment); see run.sh for the standing tasks
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u benchmarks/prefill_gemm_bench.py --ms 128,256,512,1024,2048,4096 --models qwen,llama8b --tuned > gpurun_out/geo_tuned.log 2>&1 || { tail -20 gpurun_out/geo_tuned.log; exit 1; }
tail -1 gpurun_out/geo_tuned.log
