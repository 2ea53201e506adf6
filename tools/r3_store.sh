#!/bin/bash
# Store-mode gradients: GPU tests (kernels TN, model, RCCL, graph), in-process step A/Bs.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_rccl_gpu.py tests/test_graph_gpu.py tests/test_dist_gpu.py -k "tn or model or paired or store or rccl or routing or graph or dist" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/ab_bench.py --configs "zero:JMAE_STORE_GRADS=0" "store:JMAE_STORE_GRADS=1" --rounds 6 --steps 6 > $O/ab_pre.txt 2>&1 || { tail -20 $O/ab_pre.txt; exit 1; }
grep median $O/ab_pre.txt
timeout -k 10 300 python -u tools/ab_bench.py --task finetune --configs "zero:JMAE_STORE_GRADS=0" "store:JMAE_STORE_GRADS=1" --rounds 5 --steps 10 > $O/ab_ft.txt 2>&1 || { tail -20 $O/ab_ft.txt; exit 1; }
grep median $O/ab_ft.txt
