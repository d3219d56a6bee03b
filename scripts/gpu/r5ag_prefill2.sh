# Round 5: prefill tiles with 32-deep stages on 4-deep rings: tests, warm + cold sweeps, prefill timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "prefill_wide_tiles or prefill_lds_gemm" > gpurun_out/r5ag_tests.log 2>&1 || { echo T_FAIL; tail -60 gpurun_out/r5ag_tests.log; exit 1; }
tail -1 gpurun_out/r5ag_tests.log
for c in "" "--cold"; do
timeout -k 10 400 python -u benchmarks/prefill_tile_sweep.py $c --projs gate_up,down --ms 320,448,640 --tiles 0,1024,1281,1282,2560,2561,2562,2563 --sks 0,2,3 --iters 8 >> gpurun_out/r5ag_sweep.log 2>&1 || { tail -30 gpurun_out/r5ag_sweep.log; exit 1; }
done
grep '^{' gpurun_out/r5ag_sweep.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(d['proj'], d['M'], 'cold' if d['cold'] else 'warm', 'lib', d['hipblaslt_us'], 'best', d['best'], d['best_us'], {k: v for k, v in d['all'].items() if k.endswith('/0') or k.startswith('128')})
"
timeout -k 10 300 python -u benchmarks/timeline.py --prefill --batch 8 --ctx 50 > gpurun_out/r5ag_tl_prefill.log 2>&1 || { tail -30 gpurun_out/r5ag_tl_prefill.log; exit 1; }
head -c 300 gpurun_out/r5ag_tl_prefill.log
