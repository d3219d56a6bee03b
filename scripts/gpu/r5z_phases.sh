# Round 5: phases of the fused QKV + attention launch (Qwen decode shape; 70B TP8 rank shape)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u benchmarks/qa_phases.py > gpurun_out/r5z_phases.log 2>&1 || { tail -30 gpurun_out/r5z_phases.log; exit 1; }
timeout -k 10 200 python -u benchmarks/qa_phases.py --ctx 512 >> gpurun_out/r5z_phases.log 2>&1 || { tail -30 gpurun_out/r5z_phases.log; exit 1; }
timeout -k 10 300 python -u benchmarks/qa_phases.py --hq 8 --hkv 1 --hidden 8192 --ctx 128 >> gpurun_out/r5z_phases.log 2>&1 || { tail -30 gpurun_out/r5z_phases.log; exit 1; }
grep '^{' gpurun_out/r5z_phases.log
