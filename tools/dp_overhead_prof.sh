#!/bin/bash
# rocprofv3 kernel traces of the flagship step, plain vs a 1-rank RCCL group (JMAE_FORCE_PG=1, env://
# rendezvous without torchrun so the profiled process is bench.py itself).
#   gpurun --timeout 900 -- bash tools/dp_overhead_prof.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$1; mkdir -p $O; cd /tmp
for v in plain:0 dp64:1 dp64hp:1; do
  n=${v%%:*}; f=${v##*:}
  hp=0; [ "$n" = dp64hp ] && hp=1
  JMAE_RCCL_HIPRI=$hp JMAE_FORCE_PG=$f RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541 timeout -k 10 300 \
    rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run --output-format csv -- python $R/bench.py --steps 6 --warmup 3 \
    > $O/prof_$n.log 2>&1 || { tail -20 $O/prof_$n.log; exit 1; }
  grep '^{' $O/prof_$n.log | cut -c1-200
done
