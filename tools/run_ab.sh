set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python tools/ab_bench.py --rounds 4 --steps 6 --configs "all_blas:JMAE_GEMM=blas,JMAE_DGRAD=0,JMAE_WGRAD=0" "prev:JMAE_GEMM=auto,JMAE_DGRAD=1,JMAE_WGRAD=0" "with_tn_wgrad:JMAE_GEMM=auto,JMAE_DGRAD=1,JMAE_WGRAD=1" > gpurun_out/ab.txt 2>&1; rc=$?
cat gpurun_out/ab.txt | grep -v amdgpu
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
cat gpurun_out/bench.json
