"""Model FLOP counts (matmul FLOPs, 2 per multiply-add) for images/sec -> MFU reporting.

Counts exactly the GEMM / attention work the reference model performs per image
(/root/reference/src/modeling.py:127-274, pretraining.py:76-122) with MAE's mask-first encoder:
the encoder sees 3 CLS + keep patch tokens, the decoder all 3 + N tokens.  Elementwise work is
ignored (standard MFU convention).  Training = 3 x forward (backward = 2 x forward).
"""

from __future__ import annotations

from ..config import DecoderConfig, ViTConfig

MI355X_BF16_DENSE_PEAK = 2.5e15  # FLOP/s per GPU, dense (no 2:4 sparsity)


def _block(tokens: int, dim: int, hidden: int, ff_tokens: int) -> float:
    qkv_o = 2 * tokens * dim * 4 * dim
    attn = 2 * 2 * tokens * tokens * dim
    ff = 2 * 2 * ff_tokens * dim * hidden
    return qkv_o + attn + ff


def encoder_fwd_flops(vc: ViTConfig, keep: int) -> float:
    c = vc.num_cls_tokens
    t = c + keep
    d = vc.dim
    per_layer = _block(t, d, vc.hidden_dim, keep) + 2 * 2 * (c * d) * (4 * c * d)  # + shared jumbo MLP
    embed = 2 * keep * (vc.patch_size ** 2 * 3) * d
    return vc.layers * per_layer + embed


def pretrain_fwd_flops_per_image(vc: ViTConfig, dc: DecoderConfig) -> float:
    n = (vc.image_size // vc.patch_size) ** 2
    keep = n - int(n * (vc.image_mask_ratio or 0.0))
    c = vc.num_cls_tokens
    enc = encoder_fwd_flops(vc, keep)
    proj = 2 * (c + keep) * vc.dim * dc.dec_dim
    dec = dc.dec_layers * _block(c + n, dc.dec_dim, dc.hidden_dim, c + n)
    pred = 2 * n * dc.dec_dim * (vc.patch_size ** 2 * 3)
    return enc + proj + dec + pred


def finetune_fwd_flops_per_image(vc: ViTConfig) -> float:
    n = (vc.image_size // vc.patch_size) ** 2
    enc = encoder_fwd_flops(vc, n)
    head = 2 * vc.num_cls_tokens * vc.dim * max(vc.labels, 0)
    return enc + head


def mfu(images_per_sec: float, fwd_flops_per_image: float, n_gpus: int,
        peak: float = MI355X_BF16_DENSE_PEAK) -> float:
    return images_per_sec * 3.0 * fwd_flops_per_image / (n_gpus * peak)
