set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/attn_prefill_bench.py --lens 512,2048,4096 > gpurun_out/r5an_flash.log 2>&1 || { tail -30 gpurun_out/r5an_flash.log; exit 1; }
grep '^{' gpurun_out/r5an_flash.log
