#!/bin/bash
# Narrow-kernel check: GEMM GPU tests, then the narrow 128x192 kernel vs the 256x256 kernels vs
# hipBLASLt per flagship shape (tools/gemm_nt_bench.py, interleaved, one process).
#   gpurun --timeout 900 -- bash tools/r3_gemm_narrow.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q --timeout 120 --timeout-method thread -k "gemm or small_m or tn_wgrad" > $O/pytest.log 2>&1; grep -E "passed|failed|FAILED" $O/pytest.log | tail -40
tail -1 $O/pytest.log
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py tests/test_model_gpu.py -q --timeout 200 --timeout-method thread > $O/pytest_model.log 2>&1; grep -E "passed|failed|FAILED|Error" $O/pytest_model.log | tail -20
timeout -k 10 300 python -u tools/gemm_nt_bench.py --variant 0 --only jumbo2,b_jumbo2 --kinds splitk --iters 10 --rounds 3 > $O/bench.txt 2>&1 || { tail $O/bench.txt; exit 1; }
grep -v amdgpu.ids $O/bench.txt
timeout -k 10 300 python -u tools/gemm_nt_bench.py --variant 0 --only jumbo1,b_jumbo1 --kinds fwd_gelu_d,dgrad_dmul --iters 10 --rounds 3 > $O/bench_epi.txt 2>&1 || { tail $O/bench_epi.txt; exit 1; }
grep -v amdgpu.ids $O/bench_epi.txt
