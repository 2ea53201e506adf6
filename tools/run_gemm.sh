set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
for v in 4 41 42 44 47; do
timeout -k 10 300 python tools/gemm_nt_bench.py --variant $v --kinds fwd --only enc_qkv,enc_ff1,enc_ff2,dec_ff1 > gpurun_out/gemm_abl_$v.txt 2>&1 || { cat gpurun_out/gemm_abl_$v.txt; exit 1; }
echo variant $v; grep -v relerr_none gpurun_out/gemm_abl_$v.txt | cut -c1-75
done
