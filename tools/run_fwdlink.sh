# forward Link hand-off (upper block's LN1 in the lower block's last residual pass): GPU tests + in-model A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/ > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python tools/ab_bench.py --rounds 4 --steps 6 --configs "fl0:JMAE_FWD_LINKS=0" "fl1:JMAE_FWD_LINKS=1" > gpurun_out/ab.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/ab.txt; exit $rc
