#!/bin/bash
# attention kernel tests + interleaved A/B of attn_set_remap values (tools/attn_bench.py)
#   gpurun --timeout 600 -- bash tools/attn_ab.sh <outdir> <remap values, e.g. 0,1,3>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "attn or attention" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/attn_bench.py --remap $2 --shapes dec,enc,ft > $O/bench.txt 2>&1 || { tail $O/bench.txt; exit 1; }
grep -v amdgpu.ids $O/bench.txt
