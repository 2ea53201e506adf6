set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
cat gpurun_out/bench.json
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python $R/bench.py --steps 12 --warmup 2 > $R/gpurun_out/prof_bench.log 2>&1
