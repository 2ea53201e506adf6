set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -m pytest -q -x tests/test_kernels_gpu.py -k "attention" > gpurun_out/attn_test.txt 2>&1; rc=$?; tail -3 gpurun_out/attn_test.txt
[ $rc -ne 0 ] && exit $rc
for t in 2 3; do
timeout -k 10 120 python tools/attn_bench.py --tr $t > gpurun_out/attn_tr$t.txt 2>&1 || { cat gpurun_out/attn_tr$t.txt; exit 1; }
echo "== tr $t"; grep -v amdgpu gpurun_out/attn_tr$t.txt
done
timeout -k 10 600 python tools/ab_bench.py --rounds 4 --steps 6 --configs "tr2:ATTN_TR=2" "tr3:ATTN_TR=3" > gpurun_out/ab.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/ab.txt; exit $rc
