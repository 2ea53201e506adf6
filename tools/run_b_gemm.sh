set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python tools/gemm_nt_bench.py --kinds fwd,fwd_gelu,dgrad,dgrad_gelu --only b_qkv,b_wo,b_ff1,b_ff2,b_jumbo1,b_jumbo2 --variant 12 > gpurun_out/gemm_b.txt 2>&1 || { cat gpurun_out/gemm_b.txt; exit 1; }
grep -v amdgpu gpurun_out/gemm_b.txt
timeout -k 10 900 python tools/ab_bench.py --model vit_base_patch16 --rounds 3 --steps 6 --configs "auto:" "ours:JMAE_GEMM=ours" > gpurun_out/ab_b.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/ab_b.txt; exit $rc
