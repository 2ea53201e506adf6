#!/bin/bash
# round 6: full GPU suite, product-rate (driver on JPEG shards vs bench at 512/GPU), a trace of the
# driver's steady state (H2D / augment overlap), the default bench and its kernel trace.
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/${1:-r6c}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -4 $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/product_rate.py --out $O --steps 60 > $O/product.txt 2>&1 || { tail -20 $O/product.txt; exit 1; }
tail -1 $O/product.txt
mapfile -t CMD < <(python tools/product_rate.py --out $O --steps 34 --print-cmd 2>/dev/null)
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/drvprof -o drv -- "${CMD[@]}" > $O/drvprof.log 2>&1 || { tail -20 $O/drvprof.log; exit 1; }
KT=$(find $O/drvprof -name "*kernel_trace.csv" | head -1); MT=$(find $O/drvprof -name "*memory_copy_trace.csv" | head -1)
python tools/overlap_check.py "$KT" "$MT" --last 8 > $O/overlap.json 2>&1; cat $O/overlap.json
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/benchprof -o b -- python bench.py --steps 6 --warmup 3 > $O/benchprof.log 2>&1 || { tail -20 $O/benchprof.log; exit 1; }
BT=$(find $O/benchprof -name "*kernel_trace.csv" | head -1)
python tools/trace_steps.py "$BT" --last 4 --top 40 > $O/bench_steps.txt 2>&1; head -12 $O/bench_steps.txt
rm -f $(find $O/drvprof $O/benchprof -name "*.csv" -size +20M) 2>/dev/null; true
