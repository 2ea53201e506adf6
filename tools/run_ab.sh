set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 400 python -m pytest -q -x tests/test_dist_gpu.py > gpurun_out/dg.txt 2>&1; rc=$?; tail -15 gpurun_out/dg.txt; exit $rc
