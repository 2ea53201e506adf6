# attention: padded-key masking through the accumulator init (tests + microbench)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest -q -x tests/test_kernels_gpu.py tests/test_mae_kernels_gpu.py -k "attention or attn" --timeout 120 --timeout-method thread > gpurun_out/attn_test.txt 2>&1; rc=$?; tail -3 gpurun_out/attn_test.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/attn_bench.py --shapes dec,enc,ft > gpurun_out/attn_mask.txt 2>&1 || { cat gpurun_out/attn_mask.txt; exit 1; }
grep -v amdgpu gpurun_out/attn_mask.txt
