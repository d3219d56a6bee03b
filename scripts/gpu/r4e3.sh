# Round 4 HEAD evidence (3/3): scenario report (Qwen2.5-1.5B, fresh server per scenario), Llama-3-8B baseline / cache scenarios,
# Llama-3-70B TP=1 /v1/benchmark on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u benchmarks/run_report.py --engine native --out gpurun_out/r4e3_report > gpurun_out/r4e3_report.log 2>&1 || { tail -30 gpurun_out/r4e3_report.log; exit 1; }
tail -12 gpurun_out/r4e3_report.log | cut -c1-200
timeout -k 10 600 python -u benchmarks/run_report.py --engine native --quick --model meta-llama/Meta-Llama-3-8B-Instruct --port 8140 --out gpurun_out/r4e3_report_llama8b > gpurun_out/r4e3_report_llama8b.log 2>&1 || { tail -30 gpurun_out/r4e3_report_llama8b.log; exit 1; }
tail -8 gpurun_out/r4e3_report_llama8b.log | cut -c1-200
timeout -k 10 900 python -u benchmarks/bench_endpoint.py --model meta-llama/Meta-Llama-3-70B --rounds 5 > gpurun_out/r4e3_70b.log 2>&1 || { tail -30 gpurun_out/r4e3_70b.log; exit 1; }
tail -3 gpurun_out/r4e3_70b.log | cut -c1-600
