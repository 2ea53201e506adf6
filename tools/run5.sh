cd $GRAFT_REPO_ROOT
timeout -k 10 500 python tools/gemm_bench3.py 2>&1 | grep -v amdgpu.ids
