set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err; rc2=$?
tail -5 gpurun_out/bench1.err; cat gpurun_out/bench1.json
exit $rc2
