#!/bin/bash
# Attention backward A/B on one MI355X: attention GPU tests, then tools/attn_bench.py with the
# batched backward (tr 3) and its software-pipelined form (tr 4), alternating processes.
#   gpurun --timeout 600 -- bash tools/r3_attn_ab.sh <outdir> [shapes]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/$1; mkdir -p $O; SH=${2:-dec,ft12}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for tr in 3 4 3 4; do
  echo "== tr $tr"
  timeout -k 10 100 python tools/attn_bench.py --shapes $SH --tr $tr 2>&1 | grep bwd || exit 1
done
