"""MAE-specific ops: uint8 -> normalized patches, kept-patch gather, decoder unshuffle,
masked patch MSE.

Reference: pretraining.py:90-120 (normalize, mask tokens, index_sequence, extract_patches,
norm_pix, patch_mse_loss) and utils_mae.py:51-102.  The torch versions here are the oracle
and the CPU path; on the GPU the fused HIP kernels are used.
"""

from __future__ import annotations

import torch

from ..data.constants import IMAGENET_DEFAULT_MEAN, IMAGENET_DEFAULT_STD
from ..utils.mae import extract_patches_nchw, index_sequence, patch_mse_loss
from . import _ext

_MEAN_STD_CACHE: dict = {}


def _mean_std(device):
    key = str(device)
    if key not in _MEAN_STD_CACHE:
        m = torch.tensor(IMAGENET_DEFAULT_MEAN, dtype=torch.float32, device=device).view(1, 3, 1, 1)
        s = torch.tensor(IMAGENET_DEFAULT_STD, dtype=torch.float32, device=device).view(1, 3, 1, 1)
        _MEAN_STD_CACHE[key] = (m, s)
    return _MEAN_STD_CACHE[key]


def normalize_images(images_u8: torch.Tensor) -> torch.Tensor:
    """uint8 NCHW -> ((x/255) - mean) / std, float32 NCHW."""
    m, s = _mean_std(images_u8.device)
    return (images_u8.float() / 255.0 - m) / s


def normalized_patches(images_u8: torch.Tensor, patch_size: int) -> torch.Tensor:
    """uint8 NCHW -> fp32 [B, N, p*p*3] patches of the normalized image, (ph,pw,c) order."""
    if _ext.use_hip(images_u8):
        return _ext.load().patchify_normalize(images_u8.contiguous(), patch_size)
    return extract_patches_nchw(normalize_images(images_u8), patch_size).contiguous()


def gather_patches(patches: torch.Tensor, ids_keep: torch.Tensor) -> torch.Tensor:
    return index_sequence(patches, ids_keep)


def unshuffle(y: torch.Tensor, mask_token: torch.Tensor, ids_restore: torch.Tensor,
              pos: torch.Tensor, num_cls: int) -> torch.Tensor:
    """Decoder input assembly (pretraining.py:95-106 + modeling.py:289-292).

    y: [B, C+K, d] projected encoder output; returns fp32 [B, C+N, d] =
    cat(cls, index_sequence(cat(kept, mask_token x (N-K)), ids_restore) + pos).
    """
    B, CK, d = y.shape
    N = pos.shape[0]
    K = CK - num_cls
    cls = y[:, :num_cls].float()
    img = y[:, num_cls:].float()
    full = torch.cat([img, mask_token.view(1, 1, d).expand(B, N - K, d)], 1)
    full = index_sequence(full, ids_restore) + pos.view(1, N, d)
    return torch.cat([cls, full], 1)


def norm_pix(target: torch.Tensor) -> torch.Tensor:
    mean = target.mean(-1, keepdim=True)
    var = target.var(-1, keepdim=True, unbiased=False)
    return (target - mean) / torch.sqrt(var + 1e-6)


def masked_mse(pred: torch.Tensor, target: torch.Tensor, mask: torch.Tensor, norm_pix_loss: bool,
               per_sample: bool = False) -> torch.Tensor:
    t = norm_pix(target) if norm_pix_loss else target
    if per_sample:  # mean over masked patches of each image (patch_mse_loss before the batch mean)
        per_patch = (t - pred.float()).square().mean(-1)
        return (per_patch * mask).sum(-1) / mask.sum(-1)
    return patch_mse_loss(pred.float(), t, mask)
