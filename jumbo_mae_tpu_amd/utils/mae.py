"""MAE index/patch/loss helpers (pure PyTorch; also the semantic oracle for the HIP kernels).

Parity map (reference /root/reference/src/utils_mae.py):
  mask_union/intersection/not/select ...... utils_mae.py:24-42
  no_mask / all_mask ...................... utils_mae.py:44-49
  patch_mse_loss .......................... utils_mae.py:51-64
  extract_patches / merge_patches ......... utils_mae.py:67-82
  index_sequence .......................... utils_mae.py:84-85
  random_masking .......................... utils_mae.py:88-102

Semantics kept from the reference: ``random_masking`` draws ONE uniform noise vector of
length N per call, so every image of a rank's batch shares the same permutation (quirk Q1).
``mode="per-sample"`` is an opt-in extension that draws one permutation per image.
"""

from __future__ import annotations

import torch


def mask_union(mask1: torch.Tensor, mask2: torch.Tensor) -> torch.Tensor:
    return torch.logical_or(mask1 > 0, mask2 > 0).float()


def mask_intersection(mask1: torch.Tensor, mask2: torch.Tensor) -> torch.Tensor:
    return torch.logical_and(mask1 > 0, mask2 > 0).float()


def mask_not(mask: torch.Tensor) -> torch.Tensor:
    return 1.0 - mask


def mask_select(mask: torch.Tensor, this: torch.Tensor, other: torch.Tensor | None = None) -> torch.Tensor:
    if other is None:
        other = torch.zeros((), dtype=this.dtype, device=this.device)
    if this.dim() == 3:
        mask = mask.unsqueeze(-1)
    return torch.where(mask == 0.0, this, other)


def no_mask(x: torch.Tensor) -> torch.Tensor:
    return torch.zeros(x.shape[:2], device=x.device)


def all_mask(x: torch.Tensor) -> torch.Tensor:
    return torch.ones(x.shape[:2], device=x.device)


def patch_mse_loss(output: torch.Tensor, target: torch.Tensor, valid: torch.Tensor | None = None) -> torch.Tensor:
    """mean_b[ mean_n( where(valid, mean_pix (t-o)^2, 0) ) / (sum(valid)/N) ]."""
    if valid is None:
        valid = all_mask(target)
    valid_ratio = valid.sum(-1) / valid.shape[-1]
    per_patch = (target - output).square().mean(-1)
    per_patch = torch.where(valid > 0.0, per_patch, torch.zeros_like(per_patch))
    return (per_patch.mean(-1) / valid_ratio).mean()


def extract_patches(images_nhwc: torch.Tensor, patch_size: int) -> torch.Tensor:
    """(B,H,W,C) -> (B, h*w, p*p*C) with element order (ph, pw, c)."""
    b, h, w, c = images_nhwc.shape
    h, w = h // patch_size, w // patch_size
    x = images_nhwc.reshape(b, h, patch_size, w, patch_size, c)
    x = x.permute(0, 1, 3, 2, 4, 5)
    return x.reshape(b, h * w, patch_size * patch_size * c)


def extract_patches_nchw(images_nchw: torch.Tensor, patch_size: int) -> torch.Tensor:
    """Same output as ``extract_patches`` but reading NCHW input (skips the NHWC copy)."""
    b, c, h, w = images_nchw.shape
    h, w = h // patch_size, w // patch_size
    x = images_nchw.reshape(b, c, h, patch_size, w, patch_size)
    x = x.permute(0, 2, 4, 3, 5, 1)
    return x.reshape(b, h * w, patch_size * patch_size * c)


def merge_patches(patches: torch.Tensor, patch_size: int) -> torch.Tensor:
    b, n, _ = patches.shape
    h = w = int(round(n ** 0.5))
    x = patches.reshape(b, h, w, patch_size, patch_size, -1)
    x = x.permute(0, 1, 3, 2, 4, 5)
    return x.reshape(b, h * patch_size, w * patch_size, -1)


def index_sequence(x: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    """x[:, ids, ...] for a shared 1-D ``ids`` or per-sample gather for 2-D ``ids``."""
    if ids.dim() == 1:
        return x[:, ids]
    idx = ids.reshape(*ids.shape, *([1] * (x.dim() - 2))).expand(*ids.shape, *x.shape[2:])
    return torch.gather(x, 1, idx)


def masking_ids(noise: torch.Tensor, keep_len: int):
    """From uniform noise (N,) or (B,N): ids_shuffle, ids_restore, ids_keep, mask.

    On a GPU one HIP kernel computes all of it (csrc/mae.hip mask_ids: stable ranks, one
    workgroup per row) and also hands the int32 copies the gather kernels read to ops/mae.py as
    ``ids_keep._i32`` / ``ids_restore._i32``; the torch composition below is the CPU path and the
    GPU test's oracle.  The kernel holds one row in a workgroup (N <= 1024 patches: 448 px at
    p = 16 is 784); longer rows take the torch composition."""
    if noise.is_cuda and noise.shape[-1] <= 1024:
        from ..ops import _ext  # noqa: PLC0415 (utils import without the extension)
        if _ext.use_hip(noise):
            shuffle, restore, keep32, restore32, mask = _ext.load().mask_ids(noise.float().contiguous(), keep_len)
            ids_keep = shuffle[..., :keep_len]
            ids_keep._i32 = keep32
            restore._i32 = restore32
            return shuffle, restore, ids_keep, mask
    ids_shuffle = torch.argsort(noise, dim=-1)
    ids_restore = torch.argsort(ids_shuffle, dim=-1)
    ids_keep = ids_shuffle[..., :keep_len]
    base = torch.ones(noise.shape, device=noise.device, dtype=torch.float32)
    base[..., :keep_len] = 0.0
    if noise.dim() == 1:
        mask = base[ids_restore]
    else:
        mask = torch.gather(base, -1, ids_restore)
    return ids_shuffle, ids_restore, ids_keep, mask


def random_masking(x: torch.Tensor, generator: torch.Generator | None, keep_len: int,
                   mode: str = "shared", noise: torch.Tensor | None = None,
                   padding_mask: torch.Tensor | None = None):
    """Returns (kept, mask[B,N], ids_restore) like utils_mae.py:88-102.

    ``mode="shared"`` (reference semantics): one noise vector per call/rank.
    With ``padding_mask`` ([B,N], 1 = real token) the kept rows of it are
    returned as a 4th element, matching the reference's optional
    ``padding_mask`` argument (src/utils_mae.py:88-102).
    """
    b, n, _ = x.shape
    if noise is None:
        shape = (n,) if mode == "shared" else (b, n)
        noise = torch.rand(shape, generator=generator, device=x.device if generator is None else generator.device,
                           dtype=torch.float32).to(x.device)
    ids_shuffle, ids_restore, ids_keep, mask = masking_ids(noise, keep_len)
    kept = index_sequence(x, ids_keep)
    if mask.dim() == 1:
        mask = mask.unsqueeze(0).expand(b, n)
    if padding_mask is not None:
        return kept, mask, ids_restore, index_sequence(padding_mask, ids_keep)
    return kept, mask, ids_restore
