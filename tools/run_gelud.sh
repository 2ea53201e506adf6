# saved GELU derivative (EPI_GELU_D / EPI_DMUL): tests, microbench, in-model A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/ > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gelu_epi_bench.py > gpurun_out/gelud.txt 2>&1 || { cat gpurun_out/gelud.txt; exit 1; }
grep -v amdgpu gpurun_out/gelud.txt
timeout -k 10 900 python tools/ab_bench.py --rounds 4 --steps 6 --configs "gd0:JMAE_GELU_DERIV=0" "gd1:JMAE_GELU_DERIV=1" > gpurun_out/ab.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/ab.txt; exit $rc
