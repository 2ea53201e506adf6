#!/usr/bin/env bash
# Environment setup for an MI355X node (ROCm >= 7.0, PyTorch-ROCm preinstalled).
# The reference installs jax[tpu]/flax/optax (scripts/setup.sh of antofuller/jumbo_mae_tpu);
# here the only build step is the in-tree HIP extension for gfx950.
set -euo pipefail
REPO="$(cd "$(dirname "$0")/.." && pwd)"
python3 -c "import torch; assert torch.version.hip, 'PyTorch-ROCm required'; print('torch', torch.__version__, 'hip', torch.version.hip)"
python3 -c "import msgpack, PIL, numpy" || pip install --user msgpack pillow numpy
export PYTORCH_ROCM_ARCH=${PYTORCH_ROCM_ARCH:-gfx950}
python3 -m jumbo_mae_tpu_amd.csrc.build -j "${MAX_JOBS:-16}"
python3 -c "import jumbo_mae_tpu_amd._C as C; print('HIP extension OK:', len([x for x in dir(C) if not x.startswith('_')]), 'ops')"
