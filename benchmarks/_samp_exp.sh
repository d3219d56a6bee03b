set -e
mkdir -p gpurun_out
for n in 1 4 8 32; do
  VGATE_SAMPLE_NSEG=$n timeout -k 10 120 python -c "
import sys; sys.path.insert(0,'benchmarks'); sys.path.insert(0,'.')
import micro_gpu, json
print(json.dumps({'nseg_force': $n, **micro_gpu.sampler_bench()}))" >> gpurun_out/samp_exp.log 2>&1
done
timeout -k 10 200 python benchmarks/micro_gpu.py --quick > gpurun_out/micro7.log 2>&1
