#!/bin/bash
# Round check on one MI355X (run through gpurun): GPU tests, smoke, default bench, rocprof stats.
#   gpurun --timeout 1100 -- bash tools/gpucheck.sh [tag]
# Every GPU step has its own time limit; the script stops at the first failing step.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-check}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
echo "[gpucheck] tests"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
echo "[gpucheck] smoke"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "[gpucheck] bench"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo "[gpucheck] rocprof"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 2 > $O/prof_bench.log 2>&1 \
  || { tail -20 $O/prof_bench.log; exit 1; }
echo "[gpucheck] done"
