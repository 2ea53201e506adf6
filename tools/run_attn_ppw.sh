# attention bwd2: batch elements per workgroup (bias partials in registers) -- tests, microbench, in-model A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest -q -x tests/test_kernels_gpu.py -k "attention" --timeout 120 --timeout-method thread > gpurun_out/attn_test.txt 2>&1; rc=$?; tail -3 gpurun_out/attn_test.txt
[ $rc -ne 0 ] && exit $rc
for p in 1 2 4 8 16; do
timeout -k 10 120 python tools/attn_bench.py --ppw $p --shapes enc,ft,dec > gpurun_out/attn_p$p.txt 2>&1 || { cat gpurun_out/attn_p$p.txt; exit 1; }
echo "== ppw $p"; grep -v amdgpu gpurun_out/attn_p$p.txt | grep bwd
done
timeout -k 10 900 python tools/ab_bench.py --rounds 3 --steps 6 --configs "p1:ATTN_PPW=1" "p4:ATTN_PPW=4" "p8:ATTN_PPW=8" > gpurun_out/ab.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/ab.txt; exit $rc
