# ad-hoc GPU batch (the current experiment); see run.sh for the standing tasks
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tp_gpu.py -x -v --timeout 240 --timeout-method thread -m gpu \
  -k "rccl" > gpurun_out/rccl_test.log 2>&1 || { tail -40 gpurun_out/rccl_test.log; exit 1; }
tail -3 gpurun_out/rccl_test.log
