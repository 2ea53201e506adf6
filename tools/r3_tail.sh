#!/bin/bash
# End-of-round secondary check (one MI355X): secondary BASELINE configs with kernel stats
# (tools/secondary.sh), then the flagship with HIP-graph capture and with gradient accumulation 2.
#   gpurun --timeout 1100 -- bash tools/r3_tail.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$1; mkdir -p $O; cd $R
bash tools/secondary.sh $1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --hip-graph > $O/graph.json 2> $O/graph.err || { tail -20 $O/graph.err; exit 1; }
cat $O/graph.json
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --grad-accum 2 > $O/accum2.json 2> $O/accum2.err || { tail -20 $O/accum2.err; exit 1; }
cat $O/accum2.json
echo "[r3_tail] done"
