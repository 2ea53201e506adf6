#!/bin/bash
# Short-row 4-phase tiles (224 / 192 rows): GEMM GPU tests, per-shape timing of forced tile heights
# vs the automatic choice, in-process ViT-L step A/B.  gpurun --timeout 900 -- bash tools/r3_rows.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/gemm_nt_bench.py --variant 0r256t,0r224,0r192,0t --kinds fwd,fwd_gelu_d,dgrad,dgrad_dmul \
  --only enc_wo,enc_ff1,enc_ff2,enc_qkv,dec_wo,dec_qkv,dec_ff1,b_wo,ft_wo,ft_qkv,b_ff1 --rounds 3 --iters 10 > $O/gemm_rows.txt 2>&1 || { tail -20 $O/gemm_rows.txt; exit 1; }
cat $O/gemm_rows.txt
timeout -k 10 300 python -u tools/ab_bench.py --configs "r256:GEMM_ROWS=256" "auto:GEMM_ROWS=0" --rounds 4 --steps 6 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
