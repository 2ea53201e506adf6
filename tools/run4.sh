cd $GRAFT_REPO_ROOT
for m in default rocblas tunable; do timeout -k 10 500 python tools/gemm_bench2.py $m 2>&1 | grep -v amdgpu.ids || exit 1; done
