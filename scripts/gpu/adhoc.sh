# ad-hoc GPU batch (the current experiment); see run.sh for the standing tasks
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for code in 1024 1025; do
  timeout -k 10 120 python3 -u benchmarks/probes/gemm_pmc_probe.py --code $code > gpurun_out/pmc_${code}_time.log 2>&1 || { tail -20 gpurun_out/pmc_${code}_time.log; exit 1; }
  tail -1 gpurun_out/pmc_${code}_time.log
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc_${code} -o run -- python3 -u benchmarks/probes/gemm_pmc_probe.py --code $code --reps 5 > gpurun_out/pmc_${code}.log 2>&1 || { tail -20 gpurun_out/pmc_${code}.log; exit 1; }
done
ls -R gpurun_out/pmc_1024 | head
