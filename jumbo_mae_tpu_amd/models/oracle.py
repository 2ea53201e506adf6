"""Literal fp32 PyTorch transcription of the reference forward pass over a Flax-layout tree.

This is the semantic oracle used by the test-suite: it consumes the *Flax* parameter tree
(the checkpoint schema) with Flax shapes (HWIO conv kernel, DenseGeneral
(D,H,hd) kernels, ...) and follows /root/reference/src/modeling.py and pretraining.py line by
line, with standard autograd.  Our fast model (flat store, fused ops, mask-first embedding)
must match it in loss and in every gradient leaf.
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ..data.constants import IMAGENET_DEFAULT_MEAN, IMAGENET_DEFAULT_STD
from ..utils.mae import extract_patches, index_sequence, patch_mse_loss
from ..utils.posemb import fixed_sincos2d_embeddings


def tree_to_torch(tree, requires_grad=True, dtype=torch.float64, device=None):
    if isinstance(tree, dict):
        return {k: tree_to_torch(v, requires_grad, dtype, device) for k, v in tree.items()}
    return torch.tensor(tree, dtype=dtype, device=device, requires_grad=requires_grad)


def _ln(x, p, eps=1e-6):
    mean = x.mean(-1, keepdim=True)
    var = (x - mean).square().mean(-1, keepdim=True)
    return (x - mean) / torch.sqrt(var + eps) * p["scale"] + p["bias"]


def _dense(x, p):
    return x @ p["kernel"] + p["bias"]


def _dense_general_in(x, p):  # (..., D) @ (D, H, hd) -> (..., H, hd)
    return torch.einsum("...d,dhk->...hk", x, p["kernel"]) + p["bias"]


def _attention(x, p, heads):
    q = _dense_general_in(x, p["wq"])
    k = _dense_general_in(x, p["wk"])
    v = _dense_general_in(x, p["wv"])
    hd = q.shape[-1]
    z = torch.einsum("bqhd,bkhd->bhqk", q / hd ** 0.5, k)
    z = torch.einsum("bhqk,bkhd->bqhd", torch.softmax(z, -1), v)
    return torch.einsum("bqhk,hkd->bqd", z, p["wo"]["kernel"]) + p["wo"]["bias"]


def _ff(x, p):
    return _dense(F.gelu(_dense(x, p["w1"]), approximate="tanh"), p["w2"])


def _scale(p, name):
    return p[name] if name in p else 1.0


def jumbo_layer(x, p, jumbo, heads, C=3):
    x = x + _scale(p, "scale1") * _attention(_ln(x, p["norm1"]), p["attn"], heads)
    cls, pt = x[:, :C], x[:, C:]
    b = cls.shape[0]
    cc = cls.reshape(b, -1)
    cc = _ln(cc, p["norm3"])
    cc = cc + _scale(p, "scale3") * _ff(cc, jumbo)
    pt = pt + _scale(p, "scale2") * _ff(_ln(pt, p["norm2"]), p["ff"])
    return torch.cat([cc.reshape(b, C, -1), pt], 1)


def vit_layer(x, p, heads):
    x = x + _scale(p, "scale1") * _attention(_ln(x, p["norm1"]), p["attn"], heads)
    return x + _scale(p, "scale2") * _ff(_ln(x, p["norm2"]), p["ff"])


def normalize_nhwc(images_u8, dtype=torch.float64):
    x = images_u8.permute(0, 2, 3, 1).to(dtype) / 255.0
    m = torch.tensor(IMAGENET_DEFAULT_MEAN, dtype=dtype, device=images_u8.device)
    s = torch.tensor(IMAGENET_DEFAULT_STD, dtype=dtype, device=images_u8.device)
    return (x - m) / s


def patch_embed(images_nhwc, p, posemb, patch, dim):
    wte = p["wte"]
    x = F.conv2d(images_nhwc.permute(0, 3, 1, 2), wte["kernel"].permute(3, 2, 0, 1), wte["bias"], stride=patch)
    x = x.permute(0, 2, 3, 1)  # B h w D
    if "wpe" in p:
        x = x + p["wpe"]
    else:
        x = x + posemb.to(x.device, x.dtype)
    return x.reshape(x.shape[0], -1, dim)


def mae_loss(params, images_u8, noise, *, layers, dim, heads, dec_layers, dec_dim, dec_heads,
             patch, mask_ratio, norm_pix_loss=False, posemb="sincos2d", C=3, dtype=torch.float64):
    """Reference PretrainModule.__call__ with a given masking noise (shape (N,) or (B,N)).  Runs on
    the device of ``images_u8`` in ``dtype`` (fp64 on the CPU for the parity tests; fp32 on the GPU
    as the reference of the ViT-L-width test)."""
    imgs = normalize_nhwc(images_u8, dtype)
    B, H, W, _ = imgs.shape
    g = H // patch
    m = params["model"]
    pos = fixed_sincos2d_embeddings(g, g, dim) if posemb == "sincos2d" else None
    x = patch_embed(imgs, m["embed"], pos, patch, dim)
    x = torch.cat([m["cls_tokens"].expand(B, -1, -1), x], 1)
    cls, pt = x[:, :C], x[:, C:]
    N = pt.shape[1]
    keep = int(N * (1.0 - mask_ratio))
    ids_shuffle = torch.argsort(noise, dim=-1)
    ids_restore = torch.argsort(ids_shuffle, dim=-1)
    kept = index_sequence(pt, ids_shuffle[..., :keep])
    base = torch.ones(noise.shape, dtype=imgs.dtype, device=imgs.device)
    base[..., :keep] = 0
    mask = base[ids_restore] if noise.dim() == 1 else torch.gather(base, -1, ids_restore)
    if mask.dim() == 1:
        mask = mask.expand(B, N)
    x = torch.cat([cls, kept], 1)
    for i in range(layers):
        x = jumbo_layer(x, m[f"layer_{i}"], m["jumbo_mlp"], heads, C)
    x = _ln(x, m["norm"])
    x = _dense(x, params["decoder_proj"])
    enc_cls, img = x[:, :C], x[:, C:]
    mt = params["image_mask_embedding"].expand(B, N - keep, dec_dim)
    img = index_sequence(torch.cat([img, mt], 1), ids_restore)
    dpos = fixed_sincos2d_embeddings(g, g, dec_dim).to(img.device, img.dtype).reshape(1, N, dec_dim)
    x = torch.cat([enc_cls, img + dpos], 1)
    d = params["decoder_model"]
    for j in range(dec_layers):
        x = vit_layer(x, d[f"dec_layer_{j}"], dec_heads)
    x = _ln(x, d["dec_norm"])
    out = _dense(x[:, C:], params["decoder_image_output"])
    target = extract_patches(imgs, patch)
    if norm_pix_loss:
        mean = target.mean(-1, keepdim=True)
        var = target.var(-1, keepdim=True, unbiased=False)
        target = (target - mean) / torch.sqrt(var + 1e-6)
    return patch_mse_loss(out, target, mask)


def classifier_logits(params, images_nhwc, *, layers, dim, heads, patch, posemb="learnable", C=3,
                      bn_stats=None, training=True):
    m = params["model"]
    B, H, W, _ = images_nhwc.shape
    g = H // patch
    pos = fixed_sincos2d_embeddings(g, g, dim) if posemb == "sincos2d" else None
    x = patch_embed(images_nhwc, m["embed"], pos, patch, dim)
    x = torch.cat([m["cls_tokens"].expand(B, -1, -1), x], 1)
    for i in range(layers):
        x = jumbo_layer(x, m[f"layer_{i}"], m["jumbo_mlp"], heads, C)
    x = _ln(x, m["norm"])
    x = x[:, :C].reshape(B, -1)
    head = m["head"]
    if "BatchNorm_0" in head:
        bn = head["BatchNorm_0"]
        if training:
            mean = x.mean(0)
            var = (x * x).mean(0) - mean * mean
        else:
            mean, var = bn_stats
        x = (x - mean) / torch.sqrt(var + 1e-5) * bn["scale"] + bn["bias"]
    return _dense(x, head["Dense_0"])


def flatten(tree, prefix=()):
    out = {}
    for k, v in tree.items():
        if isinstance(v, dict):
            out.update(flatten(v, prefix + (k,)))
        else:
            out["/".join(prefix + (k,))] = v
    return out


_ = math
