set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_dist_gpu.py -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/ab_bench.py --rounds 4 --steps 6 --configs "nolink:JMAE_LINK_BLOCKS=0" "link:JMAE_LINK_BLOCKS=1" > gpurun_out/ab.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/ab.txt; exit $rc
