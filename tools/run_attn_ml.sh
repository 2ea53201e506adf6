set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest -q -x tests/test_kernels_gpu.py -k "attention" --timeout 120 --timeout-method thread > gpurun_out/attn_test.txt 2>&1; rc=$?; tail -3 gpurun_out/attn_test.txt
[ $rc -ne 0 ] && exit $rc
for h in 1 2 4 8; do
timeout -k 10 120 python tools/attn_bench.py --hpw $h --shapes dec,enc,ft > gpurun_out/attn_h$h.txt 2>&1 || { cat gpurun_out/attn_h$h.txt; exit 1; }
echo "== hpw $h"; grep -v amdgpu gpurun_out/attn_h$h.txt | grep fwd
done
timeout -k 10 900 python tools/ab_bench.py --rounds 3 --steps 6 --configs "h1:ATTN_HPW=1" "h2:ATTN_HPW=2" "h4:ATTN_HPW=4" > gpurun_out/ab.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/ab.txt; exit $rc
