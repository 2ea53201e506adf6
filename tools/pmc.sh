#!/bin/bash
# rocprofv3 PMC counter passes over any benchmark program, one pass per counter group (the
# per-block limits of one pass: <= 8 SQ, <= 4 TCC, 2 GRBM), summarised by tools/pmc_summary.py:
#   gpurun --timeout 600 -- bash tools/pmc.sh <outdir> python3 tools/gemm_nt_bench.py --iters 2 ...
#   gpurun --timeout 600 -- bash tools/pmc.sh <outdir> python3 tools/attn_bench.py --iters 2 --shapes dec,enc
# The program is the direct child of rocprofv3 (no launcher in between); each pass has its own
# SIGKILL time limit (a counter request beyond the hardware's capacity hangs instead of failing).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/$1; shift; mkdir -p $O
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -d $O/p$i -o run --output-format csv -- "$@" \
    > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $O/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $(find $O -name "*counter_collection.csv") > $O/pmc.txt
cat $O/pmc.txt
