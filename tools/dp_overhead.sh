#!/bin/bash
# Cost of the data-parallel machinery itself on the flagship ViT-L step: plain process vs a 1-rank
# RCCL group (JMAE_FORCE_PG=1: bucketed async all_reduce + per-bucket optimizer), several buckets.
#   gpurun --timeout 900 -- bash tools/dp_overhead.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/$1; mkdir -p $O
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533"
run() { local n=$1; local a=$2; shift 2; (cd /tmp && timeout -k 10 240 env "$@" $R/bench.py --steps 20 --warmup 5 $a > $O/$n.json 2> $O/$n.err) \
  || { tail -20 $O/$n.err; exit 1; }; python -c "import json; d=[json.loads(l) for l in open('$O/$n.json') if l.startswith('{')][-1]; print('$n', d['ms_per_step'], d['value'], d.get('exposed_comm_ms_last_step'), d.get('reducer'), d['config']['final_loss'])"; }
run plain "" JMAE_FORCE_PG=0 python
run dp64 "" JMAE_FORCE_PG=1 JMAE_RCCL_HIPRI=0 $TR
run dp64_hipri "" JMAE_FORCE_PG=1 JMAE_RCCL_HIPRI=1 $TR
run dp64_nooverlap_hipri "--no-overlap" JMAE_FORCE_PG=1 JMAE_RCCL_HIPRI=1 $TR
run dp64_zero1_hipri "--shard-optimizer" JMAE_FORCE_PG=1 JMAE_RCCL_HIPRI=1 $TR
run dp16_hipri "--bucket-mb 16" JMAE_FORCE_PG=1 JMAE_RCCL_HIPRI=1 $TR
