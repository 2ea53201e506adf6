#!/bin/bash
# GEMM kernel A/B on the flagship shapes (tools/gemm_nt_bench.py, interleaved rounds, one process)
# plus the GEMM GPU tests first.  Variants: 0 = default routing, 1 = 64-deep main loop everywhere;
# suffix t = tail split (gemm_nt_bench.py --variant).
#   gpurun --timeout 600 -- bash tools/gemm_ab.sh <outdir> <variants> [shapes] [kinds]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/$1; mkdir -p $O
V=${2:-0}; SH=${3:-}; KI=${4:-fwd,fwd_gelu,dgrad}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k gemm > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u tools/gemm_nt_bench.py --variant $V ${SH:+--only $SH} --kinds $KI --iters 10 --rounds 3 > $O/bench.txt 2>&1 || { tail $O/bench.txt; exit 1; }
grep -v amdgpu.ids $O/bench.txt
