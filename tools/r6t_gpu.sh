#!/bin/bash
# round 6 (t): is the LayerNorm backward byte-bound?  tools/ln_bench.py paths x (fp32 input) / h (bf16 LN output + affine
# inverse) from the tree, and path h from _abc/d7 (tools/r6_diag_trees.sh d7) where the bf16 values are used as x-hat directly (no LDS loads, no
# transform: timing only)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6t; mkdir -p $O
for i in 1 2; do
  timeout -k 10 120 python -u tools/ln_bench.py --paths x,h > $O/t$i.txt 2>&1 || { tail -20 $O/t$i.txt; exit 1; }
  JMAE_ROOT=$R/_abc/d7 timeout -k 10 120 python -u _abc/d7/tools/ln_bench.py --paths h > $O/d$i.txt 2>&1 || { tail -20 $O/d$i.txt; exit 1; }
done
for f in t1 d1 t2 d2; do echo "== $f"; grep -v amdgpu.ids $O/$f.txt; done
