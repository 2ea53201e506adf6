#!/bin/bash
# round 6 (k): dropout overhead at the finetune per-GPU shape (ViT-B/16, 128 images) and a variant tree _abc/h1 whose
# dropout hash multiplies by 24-bit constants (v_mul_u32_u24, full rate) instead of v_mul_lo_u32; alternating processes
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6k; mkdir -p $O
A="--task finetune --batch-per-gpu 128 --steps 30 --warmup 5"
for i in 1 2 3; do
  timeout -k 10 200 python -u tools/bench_task.py $A --dropout 0.1 > $O/base_d$i.txt 2>&1 || { tail -20 $O/base_d$i.txt; exit 1; }
  timeout -k 10 200 python -u _abc/h1/tools/bench_task.py $A --dropout 0.1 > $O/h1_d$i.txt 2>&1 || { tail -20 $O/h1_d$i.txt; exit 1; }
  timeout -k 10 200 python -u tools/bench_task.py $A > $O/base_z$i.txt 2>&1 || { tail -20 $O/base_z$i.txt; exit 1; }
done
for f in $O/*.txt; do echo "$(basename $f) $(grep '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; done
