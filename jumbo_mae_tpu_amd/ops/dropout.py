"""Dropout with a counter-based hash mask (reference src/modeling.py:133-148, flax nn.Dropout).

The keep bit of element ``i`` is a pure function of ``(seed, i)`` (``csrc/common.h``
``drop_keep``: one 32-bit hash per pair of elements, 16-bit thresholds; :func:`keep_mask` is its
bit-exact torch mirror), so no mask is ever stored: the
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


def _hash(j: torch.Tensor, seed: int) -> torch.Tensor:
    """common.h drop_hash: lowbias32 finalizer of (j + seed_lo) ^ seed_hi, all mod 2^32."""
    s_lo, s_hi = seed & _M32, (seed >> 32) & _M32
    x = ((j + s_lo) & _M32) ^ s_hi
    x = x ^ (x >> 16)
    x = _mul32(x, 0x7FEB352D)
    x = x ^ (x >> 15)
    x = _mul32(x, 0x846CA68B)
    return x ^ (x >> 16)


def keep_threshold(rate: float) -> tuple[int, float]:
    """(16-bit keep threshold, 1/keep scale) of a drop rate in [0, 1)."""
    if not 0.0 <= rate < 1.0:
        raise ValueError(f"dropout rate must be in [0, 1), got {rate}")
    keep = 1.0 - rate
    return int(round(keep * 65536.0)), 1.0 / keep


def keep_of_index(seed: torch.Tensor, idx: torch.Tensor, rate: float) -> torch.Tensor:
    """bool: keep bits of the given int64 element indices (bit-exact mirror of common.h drop_keep:
    one hash per pair idx >> 1, its low / high 16 bits for even / odd idx)."""
    thr, _ = keep_threshold(rate)
    s = int(seed.reshape(-1)[0].item())
    h = _hash((idx >> 1) & _M32, s)
    v = torch.where((idx & 1) == 1, h >> 16, h & 0xFFFF)
    return v < thr


def keep_mask(seed: torch.Tensor, n: int, rate: float, device=None) -> torch.Tensor:
    """bool [n]: the keep bits of elements 0..n-1 (elementwise dropout sites)."""
    return keep_of_index(seed, torch.arange(n, dtype=torch.int64, device=device), rate)


def keep_mask_rows(seed: torch.Tensor, rows: int, S: int, rate: float, device=None) -> torch.Tensor:
    """bool [rows, S]: attention-probability keep bits for rows r = (b H + h) S + q: element (r, c)
    at index ((r - q) + c) * SE + q with SE = S rounded up to even -- transposed, so that queries
    2m, 2m + 1 of a key share one hash (the fused attention kernels' convention)."""
    se = S + (S & 1)
    r = torch.arange(rows, dtype=torch.int64, device=device)[:, None]
    q = r % S
    c = torch.arange(S, dtype=torch.int64, device=device)
    return keep_of_index(seed, (r - q + c) * se + q, rate)


def draw_seed(rng: torch.Generator | None, device) -> torch.Tensor:
    return torch.randint(0, 2 ** 62, (1,), generator=rng, device=device, dtype=torch.int64)


def draw_seeds(rng: torch.Generator | None, device, n: int) -> list[torch.Tensor]:
    """n seeds from ONE draw (one kernel per layer instead of one per dropout site)."""
    t = torch.randint(0, 2 ** 62, (n,), generator=rng, device=device, dtype=torch.int64)
    return [t[i:i + 1] for i in range(n)]


def _apply(x: torch.Tensor, seed: torch.Tensor, rate: float) -> torch.Tensor:
    if x.is_cuda:
        return _ext.load(True).dropout_apply(x.contiguous(), seed, rate)
    _, scale = keep_threshold(rate)
    m = keep_mask(seed, x.numel(), rate, x.device).view(x.shape)
    return torch.where(m, x * scale, torch.zeros((), dtype=x.dtype))


def apply_(x: torch.Tensor, seed: torch.Tensor, rate: float) -> torch.Tensor:
    """In place: x *= keep(seed, i) / keep over x's flat elements (the fused blocks' Dense-output
    dropout, forward on the branch output and backward on its gradient)."""
    if x.is_cuda:
        _ext.load(True).dropout_apply_(x, seed, rate)
        return x
    _, scale = keep_threshold(rate)
    m = keep_mask(seed, x.numel(), rate, x.device).view(x.shape)
    return x.mul_(m.to(x.dtype) * scale)


def gelu_drop(a: torch.Tensor, gp: torch.Tensor | None, seed: torch.Tensor, rate: float):
    """FF hidden dropout of the fused blocks -> (gelu(h) m, gelu'(h) m) with m = keep / keep_p:
    ``gp`` given: ``a`` = gelu(h) and ``gp`` = gelu'(h) (the fused epilogue's pair), masked in
    place; else ``a`` is the pre-activation h."""
    if a.is_cuda:
        g, d = _ext.load(True).gelu_drop(a, gp, seed, rate)
        return g, d
    _, scale = keep_threshold(rate)
    m = keep_mask(seed, a.numel(), rate, a.device).view(a.shape).to(torch.float32) * scale
    if gp is not None:
        a.copy_((a.float() * m).to(a.dtype))
        gp.copy_((gp.float() * m).to(gp.dtype))
        return a, gp
    x = a.float()
    t = torch.tanh(0.7978845608028654 * (x + 0.044715 * x ** 3))
    g = 0.5 * x * (1 + t)
    d = 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * x * x)
    return (g * m).to(a.dtype), (d * m).to(a.dtype)


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


def dropout(x: torch.Tensor, rate: float, rng: torch.Generator | None, seed: torch.Tensor | None = None) -> torch.Tensor:
    """Inverted dropout of ``x`` (train mode); rate 0 is the identity, rate 1 gives zeros.
    ``seed``: a pre-drawn seed (draw_seeds) instead of a draw from ``rng``."""
    if rate <= 0.0:
        return x
    if rate >= 1.0:
        return x * 0.0
    if x.is_cuda and x.numel() % 8:
        raise ValueError("dropout: the HIP kernel needs numel % 8 == 0")
    return _Dropout.apply(x, seed if seed is not None else draw_seed(rng, x.device), rate)


class _SoftmaxDropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, seed, rate):
        if z.is_cuda:
            p, pd = _ext.load(True).softmax_dropout_fwd(z, seed, rate)
        else:
            p = torch.softmax(z, -1)
            _, scale = keep_threshold(rate)
            m = keep_mask_rows(seed, z.numel() // z.shape[-1], z.shape[-1], rate, z.device).view(z.shape)
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
        m = keep_mask_rows(seed, p.numel() // p.shape[-1], p.shape[-1], ctx.rate, p.device).view(p.shape)
        dp = torch.where(m, dpd * scale, torch.zeros((), dtype=dpd.dtype))
        return p * (dp - (p * dp).sum(-1, keepdim=True)), None, None


def softmax_dropout(z: torch.Tensor, rate: float, rng: torch.Generator | None,
                    seed: torch.Tensor | None = None) -> torch.Tensor:
    """dropout(softmax(z, -1)) for fp32 logits ``z`` [..., S] (train mode)."""
    z = z.float().contiguous()
    if rate <= 0.0:
        return torch.softmax(z, -1)
    if rate >= 1.0:
        return z * 0.0
    return _SoftmaxDropout.apply(z, seed if seed is not None else draw_seed(rng, z.device), rate)
