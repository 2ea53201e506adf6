# two-build A/B of the FF GELU epilogues (abtmp/old vs the tree) + GPU tests
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/ > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
for v in old new; do
if [ $v = old ]; then PP=$R/abtmp/old; else PP=$R; fi
JMAE_ROOT=$PP timeout -k 10 200 python tools/gelu_epi_bench.py --rounds 2 > gpurun_out/epi_$v$i.txt 2>&1 || { cat gpurun_out/epi_$v$i.txt; exit 1; }
echo "== $v $i"; grep -v amdgpu gpurun_out/epi_$v$i.txt | grep dgrad
done
done
