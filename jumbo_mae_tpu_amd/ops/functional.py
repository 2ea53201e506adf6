"""Per-op autograd wrappers of the hot-path primitives (ops/prims.py).

Used for the parts of the model that are not fused transformer blocks (patch embedding,
decoder projection / prediction head, final norms, the finetune head) and as the generic path
for configurations the fused blocks do not cover (dropout > 0).  Parameter gradients never travel
through autograd: each op accumulates them straight into the flat fp32 gradient buffer of the
``ParamStore`` and signals the data-parallel reducer; parameters are passed as autograd inputs
only so that the graph records the ops that own them.

Reference semantics (file:line in /root/reference/src):
  Dense/DenseGeneral + bias ........... modeling.py:30-31,127-148
  LayerNorm (eps 1e-6, Flax default) .. modeling.py:155-156,177-179,238,282
  gelu (tanh approximation) ........... modeling.py:148 (flax nn.gelu approximate=True)
  softmax attention, no mask .......... modeling.py:135-138
  droppath = per-sample Dropout ....... modeling.py:157,181-183 (broadcast_dims)
"""

from __future__ import annotations

import torch

from ..models.params import Handle
from . import prims as P
from .prims import LN_EPS, wgrad_split  # noqa: F401  (re-exported)


# ---------------------------------------------------------------------------------- linear
class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wp, bp, hw: Handle, hb: Handle | None, gelu: bool):
        x2 = x.reshape(-1, x.shape[-1])
        if gelu:
            h, out = P.linear_gelu_fwd(x2, hw, hb)
            ctx.save_for_backward(x2, h)
        else:
            out = h = P.linear_fwd(x2, hw, hb)
            ctx.save_for_backward(x2)
        ctx.hw, ctx.hb, ctx.gelu = hw, hb, gelu
        ctx.xshape = x.shape
        ctx.x_requires_grad = x.requires_grad
        return out.reshape(*x.shape[:-1], out.shape[-1])

    @staticmethod
    def backward(ctx, dout):
        hw, hb = ctx.hw, ctx.hb
        dout = dout.reshape(-1, dout.shape[-1]).contiguous()
        bias_done = False
        if ctx.gelu:
            x2, h = ctx.saved_tensors
            dy, bias_done = P.gelu_bwd(h, dout, hb if hw.segs[0].trainable else None)
        else:
            (x2,) = ctx.saved_tensors
            dy = dout
        dx = P.linear_bwd(dy, x2, hw, hb, need_dx=ctx.x_requires_grad, bias_done=bias_done)
        if dx is not None:
            dx = dx.reshape(ctx.xshape)
        return dx, None, None, None, None, None


def linear(x: torch.Tensor, hw: Handle, hb: Handle | None = None, gelu: bool = False) -> torch.Tensor:
    hw.note_use()
    if hb is not None:
        hb.note_use()
    return _Linear.apply(x, hw.param, hb.param if hb is not None else None, hw, hb, gelu)


def gelu_fwd(h: torch.Tensor) -> torch.Tensor:
    return P.gelu_fwd(h)


def gelu_bwd(h: torch.Tensor, da: torch.Tensor) -> torch.Tensor:
    return P.gelu_bwd(h, da)[0]


# ------------------------------------------------------------------------------- layernorm
class _LayerNorm(torch.autograd.Function):
    """x: fp32 [B, T, D] (any strides, last dim contiguous) -> y [B*(T-row0), D] in ``out_dtype``,
    the LayerNorm of rows t >= row0.  With row0 > 0 the gradient of the whole x is returned
    directly -- LN' written into rows >= row0 of a fresh tensor, zeros into the few rows below --
    instead of autograd's slice backward (a full-size zero fill plus a copy of the rows)."""

    @staticmethod
    def forward(ctx, x, gp, bp, hg: Handle, hb: Handle, out_dtype, row0=0):
        y, mean, rstd = P.ln_fwd(x[:, row0:] if row0 else x, hg, hb, out_dtype)
        ctx.save_for_backward(x, mean, rstd)
        ctx.hg, ctx.hb, ctx.row0 = hg, hb, row0
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd = ctx.saved_tensors
        r0 = ctx.row0
        if not r0:
            return P.ln_bwd(dy, x, mean, rstd, ctx.hg, ctx.hb), None, None, None, None, None, None
        dx = torch.empty(x.shape, dtype=x.dtype, device=x.device)
        dx[:, :r0].zero_()
        P.ln_bwd(dy, x[:, r0:], mean, rstd, ctx.hg, ctx.hb, out=dx[:, r0:])
        return dx, None, None, None, None, None, None


def layer_norm(x: torch.Tensor, hg: Handle, hb: Handle, out_dtype=None, row0: int = 0) -> torch.Tensor:
    """LayerNorm of x (rows t >= ``row0`` of a [B, T, D] x only, when given)."""
    if x.dim() == 2:
        x = x.unsqueeze(0)
    out_dtype = out_dtype or hg.store.compute_dtype
    hg.note_use()
    hb.note_use()
    return _LayerNorm.apply(x, hg.param, hb.param, hg, hb, out_dtype, row0)


# -------------------------------------------------------------------------------- residual
class _Residual(torch.autograd.Function):
    """out[b,t,:] = x[b,t,:] + mask[b] * scale[:] * y[b*T+t, :]  (x fp32 view, out fp32 contiguous).

    ``mask`` is the per-sample droppath keep mask already divided by the keep probability
    (Flax ``Dropout(broadcast_dims=...)`` semantics), ``scale`` the LayerScale vector.
    """

    @staticmethod
    def forward(ctx, x, y, sp, hs: Handle | None, mask):
        B, T, D = x.shape
        y2 = y.reshape(B * T, D)
        out = P.residual_fwd(x, y2, hs, mask)
        ctx.save_for_backward(y2 if hs is not None else None, mask)
        ctx.hs = hs
        ctx.ydtype = y.dtype
        ctx.yshape = y.shape
        return out

    @staticmethod
    def backward(ctx, dout):
        y2, mask = ctx.saved_tensors
        dout = dout.contiguous()
        dy, _ = P.residual_bwd(dout, y2, ctx.hs, mask, ctx.ydtype)
        return dout, dy.reshape(ctx.yshape), None, None, None


def residual(x: torch.Tensor, y: torch.Tensor, hs: Handle | None = None, mask: torch.Tensor | None = None):
    if hs is not None:
        hs.note_use()
    return _Residual.apply(x, y, hs.param if hs is not None else None, hs, mask)


# ------------------------------------------------------------------------------- attention
class _Attention(torch.autograd.Function):
    """qkv: [B, S, 3, H, hd] (compute dtype) -> o: [B, S, H*hd]."""

    @staticmethod
    def forward(ctx, qkv, heads: int):
        o, lse = P.attn_fwd(qkv, heads)
        ctx.save_for_backward(qkv, o, lse)
        ctx.heads = heads
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        return P.attn_bwd(do, qkv, o, lse, ctx.heads)[0], None


def attention(qkv: torch.Tensor, heads: int) -> torch.Tensor:
    return _Attention.apply(qkv, heads)
