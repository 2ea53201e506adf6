set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
rm -rf $R/gpurun_out/apmc1 $R/gpurun_out/apmc2
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS -d $R/gpurun_out/apmc1 -o run --output-format csv -- python3 $R/tools/attn_bench.py --iters 2 --shapes dec,enc > $R/gpurun_out/apmc1.log 2>&1 || { tail -5 $R/gpurun_out/apmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LEVEL_WAVES -d $R/gpurun_out/apmc2 -o run --output-format csv -- python3 $R/tools/attn_bench.py --iters 2 --shapes dec,enc > $R/gpurun_out/apmc2.log 2>&1 || { tail -5 $R/gpurun_out/apmc2.log; exit 1; }
echo OK
