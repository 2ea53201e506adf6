#!/bin/bash
# round 6: whole-step A/B, xor-free TN loop (this tree) vs HEAD (_abbase), default bench.py alternating
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/${1:-r6g}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_tn or wgrad" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python -u _abbase/bench.py --steps 10 --warmup 3 > $O/a$i.json 2> $O/a$i.err || { tail $O/a$i.err; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/b$i.json 2> $O/b$i.err || { tail $O/b$i.err; exit 1; }
  python -c "import json;a=json.load(open('$O/a$i.json'));b=json.load(open('$O/b$i.json'));print('round $i: HEAD',a['ms_per_step'],'ms  xor-free TN',b['ms_per_step'],'ms')"
done
