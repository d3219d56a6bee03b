# Round 5: wide-N mid-M prefill tiles: tests, tile sweep at the serving buckets, prefill step timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "prefill_wide_tiles or prefill_lds_gemm" > gpurun_out/r5af_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5af_tests.log; exit 1; }
tail -1 gpurun_out/r5af_tests.log
timeout -k 10 400 python -u benchmarks/prefill_tile_sweep.py --ms 320,448,640 --tiles 0,1024,768,1280,1281,2560,2561 --sks 0,2,3 > gpurun_out/r5af_sweep.log 2>&1 || { tail -30 gpurun_out/r5af_sweep.log; exit 1; }
grep '^{' gpurun_out/r5af_sweep.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(d['proj'], d['M'], 'lib', d['hipblaslt_us'], 'auto', d['auto_us'], 'best', d['best'], d['best_us'], {k: v for k, v in d['all'].items() if k.startswith(('1024/0', '768/0', '1280/0', '2560', '2561'))})
"
timeout -k 10 300 python -u benchmarks/timeline.py --prefill --batch 8 --ctx 50 > gpurun_out/r5af_tl_prefill.log 2>&1 || { tail -30 gpurun_out/r5af_tl_prefill.log; exit 1; }
head -c 300 gpurun_out/r5af_tl_prefill.log
