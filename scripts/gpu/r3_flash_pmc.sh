# Round 3: PMC counters of the flash prefill kernel (one pass, 8 SQ counters)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pmc_flash -- python3 $R/benchmarks/attn_prefill_bench.py --lens 2048 --iters 3 > $R/gpurun_out/r3_flash_pmc.log 2>&1 || { tail -20 $R/gpurun_out/r3_flash_pmc.log; exit 1; }
f=$(find $R/gpurun_out/pmc_flash -name '*counter_collection.csv' | head -1)
python3 $R/benchmarks/pmc_summary.py $f --top 8 | tee $R/gpurun_out/r3_flash_pmc_summary.txt
