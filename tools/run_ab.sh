set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -m pytest -q -x tests/test_model_gpu.py > gpurun_out/mt.txt 2>&1; rc=$?; tail -2 gpurun_out/mt.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/ab_bench.py --rounds 4 --steps 6 --configs "no_defer:JMAE_DEFER_WGRAD=0" "defer:JMAE_DEFER_WGRAD=1" > gpurun_out/ab.txt 2>&1; rc=$?
cat gpurun_out/ab.txt | grep -v amdgpu
exit $rc
