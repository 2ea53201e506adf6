set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest -q -x tests/test_graph_gpu.py --timeout 200 --timeout-method thread > gpurun_out/graph_test.txt 2>&1; rc=$?; tail -30 gpurun_out/graph_test.txt
exit $rc
