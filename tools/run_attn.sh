set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -m pytest -q -x tests/test_kernels_gpu.py -k "attention or gelu or colsum" > gpurun_out/attn_test.txt 2>&1; rc=$?; tail -15 gpurun_out/attn_test.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/attn_bench.py --iters 20 > gpurun_out/attn_bench.txt 2>&1 || exit 1
cat gpurun_out/attn_bench.txt
