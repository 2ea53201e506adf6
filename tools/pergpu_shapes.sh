#!/bin/bash
# The per-GPU shapes of the 8-GPU configs on one MI355X: ViT-L pretrain at 512 images, ViT-B pretrain
# at 512, ViT-B finetune at 128 -- bench.py + a rocprofv3 kernel trace of each (tools/trace_steps.py):
#   gpurun --timeout 1200 -- bash tools/pergpu_shapes.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$1; mkdir -p $O; cd $R
run() {  # name, bench args
  local n=$1; shift
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  cat $O/$n.json
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_$n -o run --output-format csv -- \
    python $R/bench.py --steps 10 --warmup 3 "$@" > $O/prof_$n.log 2>&1) || { tail -20 $O/prof_$n.log; exit 1; }
}
run vitl_b512 --batch-per-gpu 512
run vitb_b512 --model vit_base_patch16 --batch-per-gpu 512
run ft_b128 --task finetune --batch-per-gpu 128
echo "[pergpu] done"
