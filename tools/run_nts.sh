set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest -q -x tests/test_kernels_gpu.py tests/test_mae_kernels_gpu.py -k "gemm_nt or gather or embed or unshuffle or patch_mse or glue" --timeout 120 --timeout-method thread > gpurun_out/gemm_test.txt 2>&1; rc=$?; tail -3 gpurun_out/gemm_test.txt
[ $rc -ne 0 ] && exit $rc
for v in 6 12; do
timeout -k 10 300 python tools/gemm_nt_bench.py --kinds fwd,fwd_gelu,dgrad_gelu --only enc_qkv,enc_ff1,enc_ff2,dec_qkv,dec_ff1,dec_ff2 --variant $v > gpurun_out/gemm_v$v.txt 2>&1 || { cat gpurun_out/gemm_v$v.txt; exit 1; }
echo "== variant $v"; grep -v amdgpu gpurun_out/gemm_v$v.txt
done
timeout -k 10 900 python tools/ab_bench.py --rounds 3 --steps 6 --configs "v6:GEMM_VARIANT=6" "v12:GEMM_VARIANT=12" > gpurun_out/ab.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/ab.txt; exit $rc
