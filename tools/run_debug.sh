# debug-build test + the kernel suites on the release build
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_debug_build_gpu.py > gpurun_out/debug_test.txt 2>&1; rc=$?; tail -5 gpurun_out/debug_test.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/ > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc
