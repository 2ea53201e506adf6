#!/bin/bash
# round 6 (j): decoder attention backward diagnostics (tree = HEAD build, _abc/d1 = bwd3 without its global
# loads, _abc/d2 = bwd3 without its compute loop; tools/r6_diag_trees.sh d1 / d2, then d3 / d4 for the second run) + device-augment bytes
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6j2; mkdir -p $O

for i in 1 2; do
  for t in base d3 d4; do
    if [ $t = base ]; then root=$R; else root=$R/_abc/$t; fi
    JMAE_ROOT=$root timeout -k 10 120 python -u tools/attn_bench.py --shapes dec2k,dec --iters 10 > $O/$t$i.txt 2>&1 || { tail -20 $O/$t$i.txt; exit 1; }
  done
done
for f in base1 d31 d41 base2 d32 d42; do echo "== $f"; grep -v amdgpu.ids $O/$f.txt; done
