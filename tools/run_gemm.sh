set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 200 python -m pytest -q -x tests/test_kernels_gpu.py -k "gemm or residual_ln" > gpurun_out/gemm_test.txt 2>&1; rc=$?; tail -3 gpurun_out/gemm_test.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gemm_nt_bench.py --kinds splitk,dgrad --only jumbo1,jumbo2 > gpurun_out/gemm_sk.txt 2>&1 || { cat gpurun_out/gemm_sk.txt; exit 1; }
cat gpurun_out/gemm_sk.txt
timeout -k 10 600 python tools/ab_bench.py --rounds 4 --steps 6 --configs "blas_jumbo:JMAE_GEMM=blas" "auto:JMAE_GEMM=auto" > gpurun_out/ab.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/ab.txt; exit $rc
