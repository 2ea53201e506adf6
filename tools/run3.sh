cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1; rc=$?
cat gpurun_out/gemm_bench.log | grep -v amdgpu.ids
exit $rc
