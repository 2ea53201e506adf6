set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -m pytest -q -x tests/test_kernels_gpu.py -k "gemm" > gpurun_out/gemm_test.txt 2>&1; rc=$?; tail -3 gpurun_out/gemm_test.txt
[ $rc -ne 0 ] && exit $rc
for v in 6 7 8 9; do
timeout -k 10 300 python tools/gemm_nt_bench.py --kinds fwd,dgrad --variant $v > gpurun_out/gemm_v$v.txt 2>&1 || { cat gpurun_out/gemm_v$v.txt; exit 1; }
echo "== variant $v"; grep total gpurun_out/gemm_v$v.txt
done
timeout -k 10 900 python tools/ab_bench.py --rounds 4 --steps 6 --configs "v6:GEMM_VARIANT=6" "v7:GEMM_VARIANT=7" "v8:GEMM_VARIANT=8" "v9:GEMM_VARIANT=9" > gpurun_out/ab.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/ab.txt; exit $rc
