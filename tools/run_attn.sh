set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 200 python tools/attn_bench.py --iters 20 > gpurun_out/attn_bench.txt 2>&1 || exit 1
cat gpurun_out/attn_bench.txt
cd /tmp
rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/pmc1 -o run --output-format csv -- python $R/tools/attn_bench.py --iters 2 > $R/gpurun_out/pmc1.log 2>&1
echo pmc1 rc=$?
