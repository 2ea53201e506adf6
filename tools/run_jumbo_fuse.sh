# jumbo LN3 dual output + fused fp32 split-K add: kernel + model GPU tests, bench, profile
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/ > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_l.json 2> gpurun_out/bench_l.err || { tail gpurun_out/bench_l.err; exit 1; }
cat gpurun_out/bench_l.json
cd /tmp
rm -rf $R/gpurun_out/prof
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python $R/bench.py --steps 12 --warmup 2 > $R/gpurun_out/prof_bench.log 2>&1 || exit 1
echo PROF_OK
