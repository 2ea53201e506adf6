# Full GPU state check: gpu test-suite, smoke, ViT-L + ViT-B bench, rocprofv3 kernel stats.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_l.json 2> gpurun_out/bench_l.err || { tail gpurun_out/bench_l.err; exit 1; }
cat gpurun_out/bench_l.json
timeout -k 10 400 python bench.py --model vit_base_patch16 --steps 20 --warmup 5 > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || { tail gpurun_out/bench_b.err; exit 1; }
cat gpurun_out/bench_b.json
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python $R/bench.py --steps 12 --warmup 2 > $R/gpurun_out/prof_bench.log 2>&1 || exit 1
echo PROF_OK
