#!/bin/bash
# Bisect of the 1-rank RCCL finetune step vs the plain step (tests/test_rccl_gpu.py): final loss of
# the ViT-B finetune bench under each reducer mode (overlapped, --no-overlap, ZeRO-1), plain runs twice (run-to-run determinism).
#   gpurun --timeout 600 -- bash tools/dp_det_check.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/$1; mkdir -p $O
A="--task finetune --gpus 1 --steps 2 --warmup 1 --batch-per-gpu 32 --bucket-mb 0.5"
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533"
run() { local n=$1; local a=$2; shift 2; (cd /tmp && timeout -k 10 200 env "$@" $R/bench.py $A $a > $O/$n.json 2> $O/$n.err) \
  || { tail -20 $O/$n.err; exit 1; }; python -c "import json; d=[json.loads(l) for l in open('$O/$n.json') if l.startswith('{')][-1]; print('$n', d['config']['final_loss'], d.get('ms_per_step'))"; }
run plain1 "" JMAE_FORCE_PG=0 python
run plain2 "" JMAE_FORCE_PG=0 python
run forced "" JMAE_FORCE_PG=1 $TR
run forced_nooverlap "--no-overlap" JMAE_FORCE_PG=1 $TR
run forced_zero1 "--shard-optimizer" JMAE_FORCE_PG=1 $TR
