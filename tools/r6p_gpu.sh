#!/bin/bash
# round 6 (p): encoder attention backward prefetching the next batch element's load burst into the staging registers
# (attn_bwd2_kernel, 236 VGPRs, still two workgroups per CU): attention GPU tests, then attn_bench tree vs _abbase
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6p; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_dropout_gpu.py -k "attn or drop" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  JMAE_ROOT=$R/_abbase timeout -k 10 120 python -u _abbase/tools/attn_bench.py --shapes enc2k,enc,ft12 --iters 10 > $O/a$i.txt 2>&1 || { tail -20 $O/a$i.txt; exit 1; }
  timeout -k 10 120 python -u tools/attn_bench.py --shapes enc2k,enc,ft12 --iters 10 > $O/b$i.txt 2>&1 || { tail -20 $O/b$i.txt; exit 1; }
done
for f in a1 b1 a2 b2; do echo "== $f"; grep -v amdgpu.ids $O/$f.txt; done
