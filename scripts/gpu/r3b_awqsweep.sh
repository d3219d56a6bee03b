# Round 3 (session 2): in-engine AWQ decode decomposition sweep (whole-step graph replays), Qwen2.5-1.5B batch 8 ctx 100
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u benchmarks/decode_sweep.py --batch 8 --ctx 100 --quantization awq --kinds qkv,o,gate_up,down > gpurun_out/r3b_awqsweep.log 2>&1 || { tail -30 gpurun_out/r3b_awqsweep.log; exit 1; }
grep '^{' gpurun_out/r3b_awqsweep.log
