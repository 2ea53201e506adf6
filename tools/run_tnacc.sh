# TN wgrad: split 0 accumulates into G (one partial slice less): GPU tests + in-model A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/ > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python tools/ab_bench.py --rounds 4 --steps 6 --configs "a0:GEMM_TN_ACC0=0" "a1:GEMM_TN_ACC0=1" > gpurun_out/ab.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/ab.txt; exit $rc
