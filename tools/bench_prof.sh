#!/bin/bash
# default bench.py run + rocprofv3 kernel-trace stats of a shorter run (one MI355X):
#   gpurun --timeout 700 -- bash tools/bench_prof.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/${1:-benchprof}; mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 2 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
echo done
