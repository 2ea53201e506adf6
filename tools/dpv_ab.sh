#!/bin/bash
# (The DPV variants were removed after this experiment, profiles/r6a_gemm_dma_placement.txt; kept as the recipe.)
# DMA-issue placement A/B of the 4-phase GEMM main loops (JMAE_NT_DPV / JMAE_TN_DPV variants of
# csrc/gemm.hip p4_mainloop and csrc/gemm_tn.hip gemm_tn4_kernel) against the baseline tree
# _abbase/ (tools/ab_tree.sh), alternating processes on one box.  GEMM tests first.
#   gpurun --timeout 1200 -- bash tools/dpv_ab.sh <outdir> [nt variants] [tn variants]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/$1; mkdir -p $O
NV=${2:-0,1,2}; TV=${3:-0,1,2,3}
SH=${SH:-enc_qkv_2k,enc_ff1_2k,enc_ff2_2k,dec_ff1_2k,dec_ff2_2k}
KI=${KI:-fwd,fwd_gelu_d,dgrad,dgrad_dmul}
TSH=${TSH:-enc_qkv_2k,enc_ff1_2k,enc_ff2_2k,dec_qkv_2k,dec_wo_2k,dec_ff1_2k}
for v in ${NV//,/ }; do
  JMAE_NT_DPV=$v JMAE_TN_DPV=$v timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 \
    --timeout-method thread -k "gemm" > $O/pytest_v$v.log 2>&1 || { echo "pytest v$v failed"; tail -30 $O/pytest_v$v.log; exit 1; }
  tail -1 $O/pytest_v$v.log
done
for i in 1 2; do
  if [ -n "$TV" ]; then
    timeout -k 10 200 python -u _abbase/tools/wgrad_bench.py --only $TSH > $O/tn_base_$i.txt 2>&1 || { echo "tn base failed"; tail $O/tn_base_$i.txt; exit 1; }
    for v in ${TV//,/ }; do
      JMAE_TN_DPV=$v timeout -k 10 200 python -u tools/wgrad_bench.py --only $TSH > $O/tn_v${v}_$i.txt 2>&1 || { echo "tn v$v failed"; tail $O/tn_v${v}_$i.txt; exit 1; }
    done
  fi
  if [ -n "$NV" ]; then
    timeout -k 10 300 python -u _abbase/tools/gemm_nt_bench.py --only $SH --kinds $KI --iters 10 --rounds 2 > $O/nt_base_$i.txt 2>&1 || { echo "nt base failed"; tail $O/nt_base_$i.txt; exit 1; }
    for v in ${NV//,/ }; do
      JMAE_NT_DPV=$v timeout -k 10 300 python -u tools/gemm_nt_bench.py --only $SH --kinds $KI --iters 10 --rounds 2 > $O/nt_v${v}_$i.txt 2>&1 || { echo "nt v$v failed"; tail $O/nt_v${v}_$i.txt; exit 1; }
    done
  fi
done
for f in $O/tn_*.txt $O/nt_*.txt; do echo "== $f"; grep -v amdgpu.ids $f | grep "ours"; done
