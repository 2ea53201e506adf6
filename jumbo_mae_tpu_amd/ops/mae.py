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


# ------------------------------------------------------------------ fused mask-first glue (GPU)
def _i32(ids: torch.Tensor) -> torch.Tensor:
    pre = getattr(ids, "_i32", None)  # written by the masking kernel (utils/mae.py masking_ids)
    if pre is not None:
        return pre
    return ids.to(torch.int32).contiguous()


def kept_patches(images_u8: torch.Tensor, ids_keep: torch.Tensor, patch_size: int, dtype) -> torch.Tensor:
    """Normalized pixels of the kept patches as the patch-embed GEMM operand [B*K, p*p*3].

    GPU: one HIP kernel reads the uint8 images directly (K1 normalize + K3 gather fused, no fp32
    patch tensor).  CPU: the torch composition (normalize -> patchify -> index_sequence)."""
    B = images_u8.shape[0]
    if _ext.use_hip(images_u8) and dtype == torch.bfloat16:
        return _ext.load().gather_patches(images_u8.contiguous(), _i32(ids_keep), patch_size)
    kept = index_sequence(normalized_patches(images_u8, patch_size), ids_keep)
    return kept.reshape(B * kept.shape[1], -1).to(dtype)


class _EmbedFinish(torch.autograd.Function):
    """x[b] = cat(cls_tokens, e[b] + pos[ids]) -> fp32 [B, C+K, D]  (modeling.py:121-124,249-257).

    Parameter gradients (cls_tokens, learnable wpe) go straight to the flat store."""

    @staticmethod
    def forward(ctx, e, cls_p, wpe_p, h_cls, h_wpe, pos, ids, B):
        D = e.shape[-1]
        C = h_cls.numel // D
        K = ids.shape[-1]
        if _ext.use_hip(e) and e.dtype == torch.bfloat16:
            out = _ext.load().embed_finish(e.contiguous(), pos, _i32(ids), h_cls.master.contiguous(), B)
        else:
            ev = e.float().view(B, K, D)
            if pos is not None:
                ev = ev + (pos[ids] if ids.dim() == 1 else pos[ids])
            out = torch.cat([h_cls.master.view(1, C, D).expand(B, C, D), ev], 1)
        ctx.h_cls, ctx.h_wpe, ctx.C, ctx.B, ctx.K = h_cls, h_wpe, C, B, K
        ctx.edtype = e.dtype
        ctx.save_for_backward(ids)
        return out

    @staticmethod
    def backward(ctx, dx):
        (ids,) = ctx.saved_tensors
        C, B, K = ctx.C, ctx.B, ctx.K
        D = dx.shape[-1]
        dpatch = dx[:, C:]
        if ctx.h_cls.segs[0].trainable:
            ctx.h_cls.accumulate_grad_rows(dx[:, :C].reshape(B, C * D))
        h = ctx.h_wpe
        if h is not None and h.segs[0].trainable:
            if ids.dim() == 1:
                h.grad.index_add_(0, ids, dpatch.sum(0))
            else:
                h.grad.index_add_(0, ids.reshape(-1), dpatch.reshape(-1, D))
            h.ready()
        de = dpatch.to(ctx.edtype).reshape(B * K, D)
        return de, None, None, None, None, None, None, None


def embed_finish(e: torch.Tensor, h_cls, h_wpe, pos: torch.Tensor | None, ids: torch.Tensor, B: int) -> torch.Tensor:
    h_cls.note_use()
    if h_wpe is not None:
        h_wpe.note_use()
        pos = h_wpe.master
    return _EmbedFinish.apply(e, h_cls.param, h_wpe.param if h_wpe is not None else None, h_cls, h_wpe,
                              pos, ids, B)


class _Unshuffle(torch.autograd.Function):
    """Decoder input assembly (K13, pretraining.py:95-106 + modeling.py:289-292) with the mask
    token's gradient (sum over masked rows) written straight into the flat store."""

    @staticmethod
    def forward(ctx, y, tok_p, h_tok, ids_restore, pos, C):
        ids32 = _i32(ids_restore)
        out = _ext.load().unshuffle_fwd(y.contiguous(), h_tok.master.reshape(-1).contiguous(), ids32,
                                        pos.contiguous(), C)
        ctx.save_for_backward(ids32)
        ctx.h_tok, ctx.C, ctx.K = h_tok, C, y.shape[1] - C
        return out

    @staticmethod
    def backward(ctx, dout):
        (ids32,) = ctx.saved_tensors
        dy, dtok_part = _ext.load().unshuffle_bwd(dout.contiguous(), ids32, ctx.C, ctx.K)
        if ctx.h_tok.segs[0].trainable:
            ctx.h_tok.accumulate_grad_rows(dtok_part)
        return dy, None, None, None, None, None


def unshuffle_fused(y: torch.Tensor, h_tok, ids_restore: torch.Tensor, pos: torch.Tensor, num_cls: int):
    """GPU path of ``unshuffle`` taking the mask-token Handle; falls back to the torch
    composition (autograd through ``param_value``) elsewhere."""
    if _ext.use_hip(y) and y.dtype == torch.bfloat16 and y.shape[-1] % 4 == 0 and y.shape[-1] <= 1024:
        h_tok.note_use()
        return _Unshuffle.apply(y, h_tok.param, h_tok, ids_restore, pos, num_cls)
    from .params_fn import param_value
    return unshuffle(y, param_value(h_tok).view(-1), ids_restore, pos, num_cls)


class _PatchMSE(torch.autograd.Function):
    """Per-patch MSE vs the (optionally per-patch normalized) target computed from uint8 pixels
    (K14): never materializes the target.  Returns fp32 [B, N]."""

    @staticmethod
    def forward(ctx, pred, images_u8, patch_size, norm_pix):
        B = images_u8.shape[0]
        pred2 = pred.reshape(-1, pred.shape[-1])
        mse = _ext.load().patch_mse_fwd(pred2, images_u8.contiguous(), patch_size, norm_pix)
        ctx.save_for_backward(pred2, images_u8)
        ctx.p, ctx.norm_pix, ctx.pshape = patch_size, norm_pix, pred.shape
        return mse.view(B, -1)

    @staticmethod
    def backward(ctx, dmse):
        pred2, images_u8 = ctx.saved_tensors
        dpred = _ext.load().patch_mse_bwd(pred2, images_u8.contiguous(), dmse.reshape(-1).contiguous().float(),
                                          ctx.p, ctx.norm_pix)
        return dpred.view(ctx.pshape), None, None, None


def patch_mse(pred: torch.Tensor, images_u8: torch.Tensor, patch_size: int, norm_pix_loss: bool) -> torch.Tensor:
    """mean_pix (target - pred)^2 per patch, [B, N] fp32 (utils_mae.py:51-64 before masking)."""
    B = images_u8.shape[0]
    if _ext.use_hip(pred) and pred.dtype == torch.bfloat16 and pred.stride(-1) == 1:
        return _PatchMSE.apply(pred, images_u8, patch_size, bool(norm_pix_loss))
    t = normalized_patches(images_u8, patch_size)
    if norm_pix_loss:
        t = norm_pix(t)
    return (t - pred.float().view(B, t.shape[1], -1)).square().mean(-1)


def masked_mean_loss(per_patch: torch.Tensor, mask: torch.Tensor, per_sample: bool = False) -> torch.Tensor:
    """patch_mse_loss (utils_mae.py:51-64) from per-patch errors: masked mean per sample, then the
    batch mean (per_sample=True returns the per-sample values)."""
    if mask.dim() == 1:
        mask = mask.unsqueeze(0).expand_as(per_patch)
    if per_sample:
        return (per_patch * mask).sum(-1) / mask.sum(-1)
    valid_ratio = mask.sum(-1) / mask.shape[-1]
    pp = torch.where(mask > 0.0, per_patch, torch.zeros_like(per_patch))
    return (pp.mean(-1) / valid_ratio).mean()


def mixed_patches(images_u8: torch.Tensor, plan: dict | None, patch_size: int, dtype) -> torch.Tensor:
    """All patches of the normalized (Mixup / CutMix blended, ``utils.mixup.Mixup.plan``) batch as
    the patch-embed GEMM operand [B*N, p*p*3].  GPU: one HIP kernel from uint8 (K19 fused with
    K1); CPU: normalize -> blend -> patchify in torch."""
    from ..utils.mixup import Mixup

    B = images_u8.shape[0]
    if _ext.use_hip(images_u8) and dtype == torch.bfloat16:
        if plan is None:
            return _ext.load().mix_patches(images_u8.contiguous(), None, None, None, patch_size)
        d = plan["dev"]
        return _ext.load().mix_patches(images_u8.contiguous(), d["perm"], d["params"], d["box"], patch_size)
    x = Mixup.mix_images(normalize_images(images_u8), plan)
    return extract_patches_nchw(x, patch_size).reshape(B * (x.shape[-1] // patch_size) ** 2, -1).to(dtype)
