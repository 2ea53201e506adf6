set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest -q -x tests/test_mae_kernels_gpu.py tests/test_dist_gpu.py tests/test_model_gpu.py --timeout 200 --timeout-method thread > gpurun_out/seg_test.txt 2>&1; rc=$?; tail -3 gpurun_out/seg_test.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python tools/ab_bench.py --rounds 3 --steps 6 --configs "cat:JMAE_SEG_WGRAD=0" "seg:JMAE_SEG_WGRAD=1" > gpurun_out/ab.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/ab.txt; exit $rc
