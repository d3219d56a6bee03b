# Round 3: the TP peer-stop timeout test alone, verbose
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 250 python -u -m pytest tests/test_tp_gpu.py -x -v -s --timeout 200 --timeout-method thread -k peer_stops 2>&1 | tee gpurun_out/r3_tp1b_tests.log
