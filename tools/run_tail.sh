set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest -q -x tests/test_kernels_gpu.py -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/tail_test.txt 2>&1; rc=$?; tail -15 gpurun_out/tail_test.txt
[ $rc -ne 0 ] && exit $rc
for t in 0 1; do
timeout -k 10 300 python tools/gemm_nt_bench.py --kinds fwd,fwd_gelu,dgrad,dgrad_gelu --only enc_qkv,enc_wo,enc_ff1,enc_ff2,dec_qkv,dec_wo,dec_ff1 --variant 12 --tail $t > gpurun_out/gemm_tail$t.txt 2>&1 || { cat gpurun_out/gemm_tail$t.txt; exit 1; }
echo "== tail $t"; grep -v amdgpu gpurun_out/gemm_tail$t.txt | cut -c1-70
done
timeout -k 10 900 python tools/ab_bench.py --rounds 3 --steps 6 --configs "t0:GEMM_TAIL=0" "t1:GEMM_TAIL=1" > gpurun_out/ab.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/ab.txt; exit $rc
