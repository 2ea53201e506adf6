set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 120 python -m pytest -q -x tests/test_kernels_gpu.py -k "gemm_tn" > gpurun_out/gemm_test.txt 2>&1; rc=$?; tail -15 gpurun_out/gemm_test.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/wgrad_bench.py > gpurun_out/wgrad.txt 2>&1 || { cat gpurun_out/wgrad.txt; exit 1; }
cat gpurun_out/wgrad.txt
