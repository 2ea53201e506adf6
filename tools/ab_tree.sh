#!/bin/bash
# Build a baseline copy of the package at a git revision into _abbase/ (git-ignored, travels with
# the gpurun snapshot) for cross-build A/Bs: the GPU-side script runs the tool of each tree
# (tools/X.py and _abbase/tools/X.py import their own tree's package), alternating, in separate
# processes on the same box (tools/xab.sh).  Run HERE (CPU), before the gpurun call:
#   bash tools/ab_tree.sh [rev, default HEAD]
set -e
REV=${1:-HEAD}
R=$(git rev-parse --show-toplevel); cd $R
rm -rf _abbase && mkdir -p _abbase
git archive "$REV" jumbo_mae_tpu_amd tools bench.py | tar -x -C _abbase
# the release extension only (the debug / asan variants are not needed for timing)
(cd _abbase && python -m jumbo_mae_tpu_amd.csrc.build --variant release > /dev/null)
ls -la _abbase/jumbo_mae_tpu_amd/_C*.so
echo "baseline $(git rev-parse --short $REV) in _abbase/"
