#!/bin/bash
# round 6 (q): HIP-graph replay vs eager at the per-GPU shapes (finetune 128, ViT-L pretrain 512), alternating processes
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6q; mkdir -p $O
F="--task finetune --batch-per-gpu 128 --steps 40 --warmup 8"
L="--batch-per-gpu 512 --steps 30 --warmup 5"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $F > $O/ft_e$i.txt 2>&1 || { tail -20 $O/ft_e$i.txt; exit 1; }
  timeout -k 10 200 python -u bench.py $F --hip-graph > $O/ft_g$i.txt 2>&1 || { tail -20 $O/ft_g$i.txt; exit 1; }
  timeout -k 10 200 python -u bench.py $L > $O/l_e$i.txt 2>&1 || { tail -20 $O/l_e$i.txt; exit 1; }
  timeout -k 10 200 python -u bench.py $L --hip-graph > $O/l_g$i.txt 2>&1 || { tail -20 $O/l_g$i.txt; exit 1; }
done
for f in $O/*.txt; do echo "$(basename $f) $(grep '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["config"].get("hip_graph"))')"; done
