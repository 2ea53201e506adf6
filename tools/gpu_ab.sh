#!/bin/bash
# Step-level interleaved A/B of runtime switches on the flagship ViT-L step, one process, one GPU
# (tools/ab_bench.py: same model, same data, rounds interleaved -> no cross-process variance).
#   gpurun --timeout 700 -- bash tools/gpu_ab.sh <outdir> "a:GEMM_GROUP=8" "b:GEMM_GROUP=4" ...
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 500 python -u tools/ab_bench.py --configs "$@" --rounds 4 --steps 6 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
tail -8 $O/ab.txt
