"""jumbo_mae_tpu_amd: MI355X-native Jumbo-ViT MAE pretraining / finetuning / linear probing.

Same capabilities as antofuller/jumbo_mae_tpu (JAX/TPU) re-designed for AMD Instinct MI355X:
PyTorch-ROCm eager autograd + hand-written CDNA4 HIP kernels (``jumbo_mae_tpu_amd._C``) +
RCCL all-reduce over xGMI, one process per GPU.
"""

__version__ = "0.1.0"

from .config import DecoderConfig, ViTConfig  # noqa: F401
