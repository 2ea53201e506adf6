set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -m pytest -q -x tests/test_kernels_gpu.py -k gemm > gpurun_out/gemm_test.txt 2>&1; rc=$?; tail -3 gpurun_out/gemm_test.txt
[ $rc -ne 0 ] && exit $rc
for v in 4 47; do
timeout -k 10 300 python tools/gemm_nt_bench.py --variant $v --kinds fwd,fwd_gelu > gpurun_out/gemm_abl_$v.txt 2>&1 || { cat gpurun_out/gemm_abl_$v.txt; exit 1; }
echo variant $v; cat gpurun_out/gemm_abl_$v.txt
done
