#!/bin/bash
# Cross-build A/B on one GPU box: run the same tool from the working tree (B) and from the
# baseline tree _abbase/ (A, built by tools/ab_tree.sh), alternating A B A B in separate processes,
# each step under its own time limit.
#   gpurun --timeout 900 -- bash tools/xab.sh <outdir> <tool.py> [tool args...]
# e.g. bash tools/xab.sh xg gemm_nt_bench.py --only enc_ff1,dec_ff1 --kinds fwd_gelu_d
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/$1; T=$2; shift 2; mkdir -p $O
[ -f _abbase/tools/$T ] || { echo "no _abbase/tools/$T (run tools/ab_tree.sh first)"; exit 1; }
for i in 1 2; do
  timeout -k 10 240 python -u _abbase/tools/$T "$@" > $O/a$i.txt 2>&1 || { echo "A$i failed"; tail -20 $O/a$i.txt; exit 1; }
  timeout -k 10 240 python -u tools/$T "$@" > $O/b$i.txt 2>&1 || { echo "B$i failed"; tail -20 $O/b$i.txt; exit 1; }
done
for f in a1 b1 a2 b2; do echo "== $f"; grep -v amdgpu.ids $O/$f.txt; done
