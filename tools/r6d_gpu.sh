#!/bin/bash
# round 6: LN backward from h (block-uniform path) -- tests, kernel A/B, step A/B
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/${1:-r6d}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k layernorm tests/test_vitl_parity_gpu.py tests/test_model_gpu.py > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/ln_bench.py --shapes dec2k,enc2k,dec,enc > $O/ln_bench.txt 2>&1 || { tail $O/ln_bench.txt; exit 1; }
grep -v amdgpu $O/ln_bench.txt
timeout -k 10 500 python -u tools/ab_bench.py --batch 2048 --configs "h:LN_FROM_H=1" "x:LN_FROM_H=0" --rounds 4 --steps 3 > $O/ab_ln.txt 2>&1 || { tail $O/ab_ln.txt; exit 1; }
tail -3 $O/ab_ln.txt
