#!/bin/bash
# Split-K jumbo-MLP GEMMs (K = 12288 / 9216) on the narrow tiles vs 256 x 256: GEMM tests on the
# narrow split path, in-process step A/Bs (pretrain ViT-L, finetune ViT-B).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 200 python -u -c "
import sys, pytest
from jumbo_mae_tpu_amd.ops import _ext
_ext.load(True).gemm_set_narrow_splitk(1)
sys.exit(pytest.main(['tests/test_kernels_gpu.py', '-k', 'splitk', '-x', '-q', '-p', 'no:cacheprovider']))
" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/ab_bench.py --configs "p4:NARROW_SPLITK=0" "narrow:NARROW_SPLITK=1" --rounds 5 --steps 6 > $O/ab_pre.txt 2>&1 || { tail -20 $O/ab_pre.txt; exit 1; }
grep median $O/ab_pre.txt
timeout -k 10 300 python -u tools/ab_bench.py --task finetune --configs "p4:NARROW_SPLITK=0" "narrow:NARROW_SPLITK=1" --rounds 5 --steps 10 > $O/ab_ft.txt 2>&1 || { tail -20 $O/ab_ft.txt; exit 1; }
grep median $O/ab_ft.txt
