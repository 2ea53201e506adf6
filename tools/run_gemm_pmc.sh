set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python tools/gemm_nt_bench.py > gpurun_out/gemm_nt.txt 2>&1; rc=$?
cat gpurun_out/gemm_nt.txt
[ $rc -ne 0 ] && exit $rc
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/gpmc1 -o run --output-format csv -- python $R/tools/gemm_nt_bench.py --only enc_ff1 --kinds fwd --iters 2 --rounds 1 > $R/gpurun_out/gpmc1.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $R/gpurun_out/gpmc2 -o run --output-format csv -- python $R/tools/gemm_nt_bench.py --only enc_ff1 --kinds fwd --iters 2 --rounds 1 > $R/gpurun_out/gpmc2.log 2>&1 || exit 1
echo pmc done
