#!/bin/bash
# round 6: gelu' codes by v_cvt_pk_u8_f32 + single bf16 rounding in the DMUL epilogue -- tests, kernel A/B vs
# _abbase, whole-step A/B vs _abbase (which also lacks the xor-free TN loop)
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/${1:-r6h}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or gelu or dropout" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python -u _abbase/tools/gemm_nt_bench.py --only enc_ff1_2k,dec_ff1_2k,enc_ff2_2k,dec_ff2_2k --kinds fwd_gelu_d,dgrad_dmul --iters 10 --rounds 2 > $O/ka$i.txt 2>&1 || { tail $O/ka$i.txt; exit 1; }
  timeout -k 10 300 python -u tools/gemm_nt_bench.py --only enc_ff1_2k,dec_ff1_2k,enc_ff2_2k,dec_ff2_2k --kinds fwd_gelu_d,dgrad_dmul --iters 10 --rounds 2 > $O/kb$i.txt 2>&1 || { tail $O/kb$i.txt; exit 1; }
done
for f in ka1 kb1 ka2 kb2; do echo "== $f"; grep "ours" $O/$f.txt | grep -v total | awk '{for(j=1;j<=NF;j++) if($j=="ours") printf "%s/%s %s  ", $1, $2, $(j+1)}'; echo; done
for i in 1 2; do
  timeout -k 10 300 python -u _abbase/bench.py --steps 10 --warmup 3 > $O/a$i.json 2> $O/a$i.err || { tail $O/a$i.err; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/b$i.json 2> $O/b$i.err || { tail $O/b$i.err; exit 1; }
  python -c "import json;a=json.load(open('$O/a$i.json'));b=json.load(open('$O/b$i.json'));print('round $i: base',a['ms_per_step'],'ms  new',b['ms_per_step'],'ms')"
done
