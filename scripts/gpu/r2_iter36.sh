set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "sample" --timeout 120 --timeout-method thread > gpurun_out/r2_s36.log 2>&1 || { echo S_FAIL; tail -40 gpurun_out/r2_s36.log; exit 1; }
tail -1 gpurun_out/r2_s36.log
for nt in 256 512 1024; do
VGATE_SAMPLE_THREADS=$nt timeout -k 10 300 python -u benchmarks/sampler_probe.py > gpurun_out/r2_sprobe36_$nt.log 2>&1 || { tail -30 gpurun_out/r2_sprobe36_$nt.log; exit 1; }
echo "threads=$nt"; grep round_launches gpurun_out/r2_sprobe36_$nt.log
done
