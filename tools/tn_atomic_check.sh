#!/bin/bash
# TN weight-gradient atomic split reduction (GEMM_TN_ATOMIC) + RCCL single-rank DP path, one MI355X:
#   gpurun --timeout 900 -- bash tools/tn_atomic_check.sh <outdir>
# 1. GPU tests of the atomic TN epilogue and of bench.py over a 1-rank RCCL group (JMAE_FORCE_PG)
# 2. interleaved step A/B of the atomic modes on the flagship ViT-L step (tools/ab_bench.py)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "tn_wgrad" > $O/pytest_tn.log 2>&1 || { tail -30 $O/pytest_tn.log; exit 1; }
tail -2 $O/pytest_tn.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_rccl_gpu.py \
  > $O/pytest_rccl.log 2>&1 || { tail -40 $O/pytest_rccl.log; exit 1; }
tail -6 $O/pytest_rccl.log
timeout -k 10 500 python -u tools/ab_bench.py --configs "base:GEMM_TN_ATOMIC=0" "at1:GEMM_TN_ATOMIC=1" \
  "at3:GEMM_TN_ATOMIC=3" --rounds 4 --steps 6 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
tail -8 $O/ab.txt
# where the step's D2D copies (__amd_rocclr_copyBuffer) and torch fills come from
JMAE_PROF_STACK="aten::copy_,aten::clone,aten::cat,aten::fill_,aten::zero_,aten::contiguous" timeout -k 10 300 \
  python bench.py --steps 3 --warmup 2 --profile-steps 1 > $O/prof_stack.txt 2>&1 || { tail -20 $O/prof_stack.txt; exit 1; }
grep " <- " $O/prof_stack.txt > $O/stacks.txt || true
head -c 6000 $O/stacks.txt
