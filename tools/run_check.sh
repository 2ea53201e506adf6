# GPU check: selected tests (TESTS env, default: whole gpu suite), ViT-L bench, optional rocprofv3 stats (PROF=1).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
T=${TESTS:-tests/}
timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_l.json 2> gpurun_out/bench_l.err || { tail gpurun_out/bench_l.err; exit 1; }
cat gpurun_out/bench_l.json
if [ "${BENCHB:-0}" = 1 ]; then
timeout -k 10 400 python bench.py --model vit_base_patch16 --steps 20 --warmup 5 > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || { tail gpurun_out/bench_b.err; exit 1; }
cat gpurun_out/bench_b.json
fi
if [ "${PROF:-0}" = 1 ]; then
cd /tmp
rm -rf $R/gpurun_out/prof
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python $R/bench.py --steps 12 --warmup 2 > $R/gpurun_out/prof_bench.log 2>&1 || exit 1
echo PROF_OK
fi
