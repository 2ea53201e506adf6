#!/bin/bash
# round 6 (o): where the encoder attention backward's time goes -- attn_bwd2_kernel<64,64> at the 2048-image micro-batch;
# _abc/d5 = no global loads, _abc/d6 = no compute loop (tools/r6_diag_trees.sh d5 / d6)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6o; mkdir -p $O
for i in 1 2; do
  for t in base d5 d6; do
    if [ $t = base ]; then root=$R; else root=$R/_abc/$t; fi
    JMAE_ROOT=$root timeout -k 10 120 python -u tools/attn_bench.py --shapes enc2k,enc --iters 10 > $O/$t$i.txt 2>&1 || { tail -20 $O/$t$i.txt; exit 1; }
  done
done
for f in base1 d51 d61 base2 d52 d62; do echo "== $f"; grep -v amdgpu.ids $O/$f.txt; done
