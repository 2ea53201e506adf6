#!/bin/bash
# rocprofv3 PMC passes over the fused attention kernels (tools/attn_bench.py), one pass per
# counter group (the per-block counter limits of one pass), summarised by tools/pmc_summary.py
#   gpurun --timeout 600 -- bash tools/attn_pmc.sh <outdir> [shapes, default dec,enc]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/$1; mkdir -p $O
SH=${2:-dec,enc}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o run --output-format csv -- python3 tools/attn_bench.py --iters 2 --shapes $SH \
    > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $O/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $(find $O -name "*counter_collection.csv") > $O/pmc.txt
cat $O/pmc.txt
