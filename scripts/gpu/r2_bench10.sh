set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench10_$i.json.log 2>&1 || { tail -20 gpurun_out/r2_bench10_$i.json.log; exit 1; }
tail -1 gpurun_out/r2_bench10_$i.json.log
done
