#!/bin/bash
# round 6 (v): LayerNorm backward with vs without the (default-off) h path compiled into the kernel -- the h path's
# second row-loop instantiation raises the production kernel from 152 to 160 VGPRs; tools/ln_bench.py path x,
# tree vs _abc/noh (use_h forced false), alternating processes
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6v; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/ln_bench.py --paths x > $O/t$i.txt 2>&1 || { tail -20 $O/t$i.txt; exit 1; }
  JMAE_ROOT=$R/_abc/noh timeout -k 10 120 python -u _abc/noh/tools/ln_bench.py --paths x > $O/n$i.txt 2>&1 || { tail -20 $O/n$i.txt; exit 1; }
done
for f in t1 n1 t2 n2 t3 n3; do echo "== $f"; grep -v amdgpu.ids $O/$f.txt; done
