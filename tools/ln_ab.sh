#!/bin/bash
# LayerNorm kernel tests + in-process step A/B of the LN backward variants (ln_set_bwd_la)
#   gpurun --timeout 900 -- bash tools/ln_ab.sh <outdir> "a:LN_BWD_LA=2" "b:LN_BWD_LA=3"
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "layernorm or attention" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python -u tools/ab_bench.py --configs "$@" --rounds 4 --steps 6 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
tail -8 $O/ab.txt
