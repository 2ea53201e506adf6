"""Dropout with a counter-based hash mask (reference src/modeling.py:133-148, flax nn.Dropout).

The keep bit of element ``i`` is a pure function of ``(seed, i)`` (``csrc/dropout.hip``
``keep_bit``; :func:`keep_mask` is its bit-exact torch mirror), so no mask is ever stored: the
backward regenerates it, and so does the recompute of an activation-checkpointed layer (which
redraws the same seed from the restored generator).  The seed is an int64 [1] tensor drawn from
the caller's ``torch.Generator`` on the data's device -- no host round trip, HIP-graph safe.

* :func:`dropout` -- elementwise (FF hidden / output, attention output); its backward is the same
  op on the incoming gradient.
* :func:`softmax_dropout` -- row softmax of fp32 attention logits with dropout on the
  probabilities, one fused pass each way (the backward folds the mask, the 1/keep scale and the
  softmax Jacobian into one row kernel).

On a GPU tensor both run the HIP kernels and fail loudly if the extension is missing; on CPU
they run the torch mirror (same masks bit for bit).
"""

from __future__ import annotations

import torch

from . import _ext

_M32 = 0xFFFFFFFF


def _mul32(a: torch.Tensor, c: int) -> torch.Tensor:
    """(a * c) mod 2^32 for 0 <= a, c < 2^32 in int64 without overflow (16-bit split of c)."""
    hi, lo = c >> 16, c & 0xFFFF
    return ((((a * hi) & 0xFFFF) << 16) + a * lo) & _M32


def _fmix32(h: torch.Tensor) -> torch.Tensor:
    h = h ^ (h >> 16)
    h = _mul32(h, 0x85EBCA6B)
    h = h ^ (h >> 13)
    h = _mul32(h, 0xC2B2AE35)
    return h ^ (h >> 16)


def keep_threshold(rate: float) -> tuple[int, float]:
    if not 0.0 <= rate < 1.0:
        raise ValueError(f"dropout rate must be in [0, 1), got {rate}")
    keep = 1.0 - rate
    return int(round(keep * 16777216.0)), 1.0 / keep


def keep_mask(seed: torch.Tensor, n: int, rate: float, device=None) -> torch.Tensor:
    """bool [n]: the keep bits of elements 0..n-1 (bit-exact mirror of csrc/dropout.hip keep_bit)."""
    thr, _ = keep_threshold(rate)
    s = int(seed.reshape(-1)[0].item())
    s_lo, s_hi = s & _M32, (s >> 32) & _M32
    i = torch.arange(n, dtype=torch.int64, device=device)
    h = _fmix32(((i >> 32) + s_lo) & _M32)
    h = _fmix32((i & _M32) ^ h)
    h = _fmix32((h + s_hi) & _M32)
    return (h >> 8) < thr


def draw_seed(rng: torch.Generator | None, device) -> torch.Tensor:
    return torch.randint(0, 2 ** 62, (1,), generator=rng, device=device, dtype=torch.int64)


def _apply(x: torch.Tensor, seed: torch.Tensor, rate: float) -> torch.Tensor:
    if x.is_cuda:
        return _ext.load(True).dropout_apply(x.contiguous(), seed, rate)
    _, scale = keep_threshold(rate)
    m = keep_mask(seed, x.numel(), rate, x.device).view(x.shape)
    return torch.where(m, x * scale, torch.zeros((), dtype=x.dtype))


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, seed, rate):
        ctx.save_for_backward(seed)
        ctx.rate = rate
        return _apply(x, seed, rate)

    @staticmethod
    def backward(ctx, dy):
        (seed,) = ctx.saved_tensors
        return _apply(dy, seed, ctx.rate), None, None


def dropout(x: torch.Tensor, rate: float, rng: torch.Generator | None) -> torch.Tensor:
    """Inverted dropout of ``x`` (train mode); rate 0 is the identity, rate 1 gives zeros."""
    if rate <= 0.0:
        return x
    if rate >= 1.0:
        return x * 0.0
    if x.is_cuda and x.numel() % 8:
        raise ValueError("dropout: the HIP kernel needs numel % 8 == 0")
    return _Dropout.apply(x, draw_seed(rng, x.device), rate)


class _SoftmaxDropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, seed, rate):
        if z.is_cuda:
            p, pd = _ext.load(True).softmax_dropout_fwd(z, seed, rate)
        else:
            p = torch.softmax(z, -1)
            _, scale = keep_threshold(rate)
            m = keep_mask(seed, z.numel(), rate, z.device).view(z.shape)
            pd = torch.where(m, p * scale, torch.zeros((), dtype=p.dtype))
        ctx.save_for_backward(p, seed)
        ctx.rate = rate
        return pd

    @staticmethod
    def backward(ctx, dpd):
        p, seed = ctx.saved_tensors
        dpd = dpd.contiguous()
        if p.is_cuda:
            return _ext.load(True).softmax_dropout_bwd(dpd, p, seed, ctx.rate), None, None
        _, scale = keep_threshold(ctx.rate)
        m = keep_mask(seed, p.numel(), ctx.rate, p.device).view(p.shape)
        dp = torch.where(m, dpd * scale, torch.zeros((), dtype=dpd.dtype))
        return p * (dp - (p * dp).sum(-1, keepdim=True)), None, None


def softmax_dropout(z: torch.Tensor, rate: float, rng: torch.Generator | None) -> torch.Tensor:
    """dropout(softmax(z, -1)) for fp32 logits ``z`` [..., S] (train mode)."""
    z = z.float().contiguous()
    if rate <= 0.0:
        return torch.softmax(z, -1)
    if rate >= 1.0:
        return z * 0.0
    return _SoftmaxDropout.apply(z, draw_seed(rng, z.device), rate)
