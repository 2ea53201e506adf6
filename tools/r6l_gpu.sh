#!/bin/bash
# round 6 (l): kernel traces of the finetune per-GPU shape (ViT-B/16, 128 images) at dropout 0 and 0.1
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/r6l; mkdir -p $O
A="--task finetune --batch-per-gpu 128 --steps 12 --warmup 4"
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/z -o run --output-format csv -- python $R/bench.py $A > $O/z.log 2>&1 || { tail -20 $O/z.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/d -o run --output-format csv -- python $R/bench.py $A --dropout 0.1 > $O/d.log 2>&1 || { tail -20 $O/d.log; exit 1; }
ls -R $O | head
