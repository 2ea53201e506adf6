#!/bin/bash
# Grouped segmented jumbo weight gradients: TN / model GPU tests, in-process step A/B.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -k "paired" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/ab_bench.py --configs "blocks:JMAE_GROUP_JUMBO_WGRAD=0" "blocks+jumbo:JMAE_GROUP_JUMBO_WGRAD=1" --rounds 6 --steps 6 > $O/ab_pre.txt 2>&1 || { tail -20 $O/ab_pre.txt; exit 1; }
grep median $O/ab_pre.txt
