# LN backward: early residual-gradient load (LN_BWD_LA=2) vs default (0): tests + in-model A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest -q -x tests/test_kernels_gpu.py -k "layernorm" --timeout 120 --timeout-method thread > gpurun_out/ln_test.txt 2>&1; rc=$?; tail -3 gpurun_out/ln_test.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python tools/ab_bench.py --rounds 4 --steps 6 --configs "la0:LN_BWD_LA=0" "la2:LN_BWD_LA=2" > gpurun_out/ab.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/ab.txt; exit $rc
