#!/bin/bash
# 8-wave hd-64 attention backward check: attention GPU tests, then attn_bench ft12 with the
# 8-wave (nw8 1) and 4-wave (nw8 0) batched backward alternating, then the finetune bench.
#   gpurun --timeout 700 -- bash tools/r3_attn_nw8.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for v in 1 0 1 0; do
  echo "== nw8 $v"
  timeout -k 10 100 python tools/attn_bench.py --shapes ft12,ft --nw8 $v 2>&1 | grep bwd || exit 1
done
timeout -k 10 300 python bench.py --task finetune --steps 20 --warmup 5 > $O/ft.json 2> $O/ft.err || { tail -20 $O/ft.err; exit 1; }
cat $O/ft.json
