#!/bin/bash
# Secondary BASELINE configs (bench.py --task finetune / --model vit_base_patch16 / --task linear) + a rocprofv3
# kernel-stats profile of each, on one MI355X:
#   gpurun --timeout 900 -- bash tools/secondary.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$1; mkdir -p $O; cd $R
run() {  # name, bench args
  local n=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  cat $O/$n.json
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run --output-format csv -- \
    python $R/bench.py --steps 6 --warmup 2 "$@" > $O/prof_$n.log 2>&1) || { tail -20 $O/prof_$n.log; exit 1; }
}
run finetune --task finetune
run vitb_pretrain --model vit_base_patch16
run linear --task linear
echo "[secondary] done"
