set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python $R/bench.py --steps 4 --warmup 2 > $R/gpurun_out/prof_bench.log 2>&1; rc2=$?
tail -3 $R/gpurun_out/prof_bench.log
ls -R $R/gpurun_out/prof | head
exit $rc2
