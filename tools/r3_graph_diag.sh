#!/bin/bash
# Graph-replay gradient diagnosis under the gradient-path switches (one MI355X).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/ggd; mkdir -p $O
run() { timeout -k 10 120 "$@" >> $O/log.txt 2>&1 || { echo "FAILED: $*" >> $O/log.txt; tail -30 $O/log.txt; exit 1; }; }
run python -u tools/graph_grad_diag.py --order eager_first
run python -u tools/graph_grad_diag.py --order graph_first
JMAE_STORE_GRADS=0 run python -u tools/graph_grad_diag.py --order graph_first
JMAE_PAIR_WGRAD=0 run python -u tools/graph_grad_diag.py --order graph_first
JMAE_STORE_GRADS=0 JMAE_PAIR_WGRAD=0 run python -u tools/graph_grad_diag.py --order graph_first
grep -v amdgpu.ids $O/log.txt
