# Round 3, call 1: calibrate this box (driver bench at HEAD), in-engine decode-GEMM decomposition sweep
# with the wider candidate lists, launch timeline of one decode step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_s1_bench.log 2>&1 || { tail -30 gpurun_out/r3_s1_bench.log; exit 1; }
tail -1 gpurun_out/r3_s1_bench.log | cut -c1-600
timeout -k 10 600 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --kinds down,gate_up,o,qkv > gpurun_out/r3_s1_sweep.log 2>&1 || { tail -30 gpurun_out/r3_s1_sweep.log; exit 1; }
tail -3 gpurun_out/r3_s1_sweep.log
timeout -k 10 300 python -u benchmarks/timeline.py --batch 8 --ctx 100 > gpurun_out/r3_s1_timeline.log 2>&1 || { tail -30 gpurun_out/r3_s1_timeline.log; exit 1; }
tail -2 gpurun_out/r3_s1_timeline.log | cut -c1-300
