set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
SHAPE=${SHAPE:-enc_ff1}
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/gpmc1 -o run --output-format csv -- python $R/tools/gemm_nt_bench.py --only $SHAPE --kinds fwd --iters 2 --rounds 1 > $R/gpurun_out/gpmc1.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $R/gpurun_out/gpmc2 -o run --output-format csv -- python $R/tools/gemm_nt_bench.py --only $SHAPE --kinds fwd --iters 2 --rounds 1 > $R/gpurun_out/gpmc2.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $R/gpurun_out/gpmc3 -o run --output-format csv -- python $R/tools/gemm_nt_bench.py --only $SHAPE --kinds fwd --iters 2 --rounds 1 > $R/gpurun_out/gpmc3.log 2>&1 || exit 1
cd $R && python tools/pmc_summary.py gpurun_out/gpmc1/run_counter_collection.csv gpurun_out/gpmc2/run_counter_collection.csv gpurun_out/gpmc3/run_counter_collection.csv > gpurun_out/gpmc_summary.txt
echo pmc done
