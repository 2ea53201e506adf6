#!/bin/bash
# round 6: TN weight-gradient loop without v_xor (precomputed block addresses) vs the round-5 loop (_abbase)
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/${1:-r6f}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_tn" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TSH=enc_qkv_2k,enc_wo_2k,enc_ff1_2k,enc_ff2_2k,dec_qkv_2k,dec_wo_2k,dec_ff1_2k,dec_ff2_2k
for i in 1 2; do
  timeout -k 10 200 python -u _abbase/tools/wgrad_bench.py --only $TSH > $O/a$i.txt 2>&1 || { tail $O/a$i.txt; exit 1; }
  timeout -k 10 200 python -u tools/wgrad_bench.py --only $TSH > $O/b$i.txt 2>&1 || { tail $O/b$i.txt; exit 1; }
done
for f in a1 b1 a2 b2; do echo "== $f"; grep "ours" $O/$f.txt | awk '{print $1, $9, $10, $11}' | tr '\n' ' '; echo; done
