set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or decode or engine or graph" > gpurun_out/r5ap.log 2>&1 || { tail -40 gpurun_out/r5ap.log; exit 1; }
tail -1 gpurun_out/r5ap.log
