# ad-hoc GPU batch: same-box A/B of the long-chunk tuner margin (A = 0.05 as before, B = 0.02)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
for arm in 0.05 0.02; do
timeout -k 10 400 python -u -c "
import runpy, sys
import vgate.ops as o
o.LONG_MARGIN = $arm
sys.argv = ['ttft_probe.py', '--model', 'meta-llama/Meta-Llama-3-8B-Instruct', '--lens', '2048']
runpy.run_path('benchmarks/ttft_probe.py', run_name='__main__')
" > gpurun_out/sk11_ttft_${arm}_$i.log 2>&1 || { tail -30 gpurun_out/sk11_ttft_${arm}_$i.log; exit 1; }
echo "margin $arm run $i: $(grep '^{' gpurun_out/sk11_ttft_${arm}_$i.log | tail -1)"
done
done
