set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python tools/gemm_nt_bench.py --kinds dgrad_gelu,dgrad > gpurun_out/gemm_dg.txt 2>&1 || { cat gpurun_out/gemm_dg.txt; exit 1; }
cat gpurun_out/gemm_dg.txt
