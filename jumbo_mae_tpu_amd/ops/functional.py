"""Autograd ops of the Jumbo-MAE hot path.

Every op has two implementations behind one ``torch.autograd.Function``:

* the HIP path (tensors on the MI355X): fused CDNA4 kernels from ``jumbo_mae_tpu_amd._C``
  plus hipBLASLt GEMMs (bias epilogue, bf16 in / fp32 out for weight gradients);
* the torch path (CPU): plain fp32 PyTorch that transcribes the reference math -- it is the
  numerical oracle the kernels are tested against.

Parameter gradients never travel through autograd: each op accumulates them directly into
the flat fp32 gradient buffer of the ``ParamStore`` (see models/params.py) and signals the
data-parallel reducer that the segment is ready.  Parameters are still passed as autograd
inputs so that the graph records every op that owns parameters.

Reference semantics (file:line in /root/reference/src):
  Dense/DenseGeneral + bias ........... modeling.py:30-31,127-148
  LayerNorm (eps 1e-6, Flax default) .. modeling.py:155-156,177-179,238,282
  gelu (tanh approximation) ........... modeling.py:148 (flax nn.gelu approximate=True)
  softmax attention, no mask .......... modeling.py:135-138
  droppath = per-sample Dropout ....... modeling.py:157,181-183 (broadcast_dims)
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import _ext
from ..models.params import Handle

LN_EPS = 1e-6


def _hip(t: torch.Tensor) -> bool:
    return _ext.use_hip(t)


def wgrad_split(M: int, N: int, K: int) -> int:
    """Split-K factor for a weight-gradient GEMM (reduction over M tokens, N x K output).

    The output of a wgrad is small (0.25-38 M elements) while the reduction is 25k-100k long, so a
    single GEMM has only 4-200 256x256 output tiles for 256 CUs (measured 160-690 TF/s on MI355X,
    profiles/r1_gemm_wgrad_alternatives.log).  Splitting M into S chunks of one strided-batched
    GEMM gives S x tiles workgroups (fp32 partials, reduced after): ~4x tiles-per-CU target."""
    tiles = max(1, (N // 256) * (K // 256))
    s = 1
    while s < 16 and tiles * s * 2 <= 256 and M % (s * 2) == 0 and M // (s * 2) >= 2048:
        s *= 2
    return s


def _gemm_wgrad(h: Handle, dy: torch.Tensor, x: torch.Tensor) -> None:
    """grad[h] += dy^T @ x  (fp32 accumulate; bf16 inputs on GPU)."""
    g = h.grad
    if dy.is_cuda and dy.dtype != torch.float32:
        M, N = dy.shape
        K = x.shape[1]
        s = wgrad_split(M, N, K)
        if s > 1:
            part = torch.bmm(dy.view(s, M // s, N).transpose(1, 2), x.view(s, M // s, K), out_dtype=torch.float32)
            if _hip(part):
                _ext.load().splitk_reduce_add(part, g)  # g += sum_s part[s], one fused pass
            else:
                g.add_(part.sum(0))
        else:
            torch.addmm(g, dy.t(), x, out_dtype=torch.float32, out=g)
    else:
        g.addmm_(dy.t().float(), x.float())


def _bias_grad(h: Handle | None, dy: torch.Tensor) -> None:
    if h is None:
        return
    h.grad.add_(dy.sum(0, dtype=torch.float32))


# ---------------------------------------------------------------------------------- linear
class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wp, bp, hw: Handle, hb: Handle | None, gelu: bool):
        w = hw.weight()
        x2 = x.reshape(-1, x.shape[-1])
        if hb is not None:
            h = torch.addmm(hb.weight(), x2, w.t())
        else:
            h = x2 @ w.t()
        if gelu:
            a = gelu_fwd(h)
            ctx.save_for_backward(x2, h)
            out = a
        else:
            ctx.save_for_backward(x2)
            out = h
        ctx.hw, ctx.hb, ctx.gelu = hw, hb, gelu
        ctx.xshape = x.shape
        ctx.x_requires_grad = x.requires_grad
        return out.reshape(*x.shape[:-1], out.shape[-1])

    @staticmethod
    def backward(ctx, dout):
        hw, hb = ctx.hw, ctx.hb
        dout = dout.reshape(-1, dout.shape[-1])
        trainable = hw.segs[0].trainable
        bias_fused = False
        if ctx.gelu:
            x2, h = ctx.saved_tensors
            if _hip(h):
                # dh = da * gelu'(h) with the bias gradient column-sum fused into the same pass
                bg = hb.grad if (hb is not None and trainable) else None
                dy = _ext.load().gelu_bwd(h, dout.contiguous(), bg)
                bias_fused = True
            else:
                dy = gelu_bwd(h, dout)
        else:
            (x2,) = ctx.saved_tensors
            dy = dout.contiguous()
        dx = None
        if ctx.x_requires_grad:
            dx = (dy @ hw.weight()).reshape(ctx.xshape)
        if trainable:
            _gemm_wgrad(hw, dy, x2)
            hw.ready()
            if hb is not None:
                if not bias_fused:
                    if _hip(dy):
                        _ext.load().colsum(dy, hb.grad)
                    else:
                        _bias_grad(hb, dy)
                hb.ready()
        return dx, None, None, None, None, None


def linear(x: torch.Tensor, hw: Handle, hb: Handle | None = None, gelu: bool = False) -> torch.Tensor:
    hw.note_use()
    if hb is not None:
        hb.note_use()
    return _Linear.apply(x, hw.param, hb.param if hb is not None else None, hw, hb, gelu)


# ------------------------------------------------------------------------------------ gelu
_GELU_C = math.sqrt(2.0 / math.pi)


def gelu_fwd(h: torch.Tensor) -> torch.Tensor:
    if _hip(h):
        return _ext.load().gelu_fwd(h)
    return F.gelu(h, approximate="tanh")


def gelu_bwd(h: torch.Tensor, da: torch.Tensor) -> torch.Tensor:
    if _hip(h):
        return _ext.load().gelu_bwd(h, da.contiguous())
    hf = h.float()
    u = _GELU_C * (hf + 0.044715 * hf ** 3)
    t = torch.tanh(u)
    d = 0.5 * (1 + t) + 0.5 * hf * (1 - t * t) * _GELU_C * (1 + 3 * 0.044715 * hf * hf)
    return (da.float() * d).to(h.dtype)


# ------------------------------------------------------------------------------- layernorm
class _LayerNorm(torch.autograd.Function):
    """x: fp32 [B, T, D] (any strides, last dim contiguous) -> y [B*T, D] in ``out_dtype``."""

    @staticmethod
    def forward(ctx, x, gp, bp, hg: Handle, hb: Handle, out_dtype):
        B, T, D = x.shape
        if _hip(x):
            y, mean, rstd = _ext.load().layernorm_fwd(x, hg.master, hb.master, LN_EPS, out_dtype)
        else:
            xf = x.reshape(B * T, D).float()
            mean = xf.mean(-1)
            var = (xf - mean[:, None]).square().mean(-1)
            rstd = torch.rsqrt(var + LN_EPS)
            y = ((xf - mean[:, None]) * rstd[:, None] * hg.master + hb.master).to(out_dtype)
        ctx.save_for_backward(x, mean, rstd)
        ctx.hg, ctx.hb = hg, hb
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd = ctx.saved_tensors
        hg, hb = ctx.hg, ctx.hb
        B, T, D = x.shape
        dy = dy.contiguous()
        if _hip(x):
            dx = _ext.load().layernorm_bwd(dy, x, mean, rstd, hg.master, hg.grad, hb.grad,
                                           hg.segs[0].trainable)
        else:
            xf = x.reshape(B * T, D).float()
            xhat = (xf - mean[:, None]) * rstd[:, None]
            dyf = dy.float()
            if hg.segs[0].trainable:
                hg.grad.add_((dyf * xhat).sum(0))
                hb.grad.add_(dyf.sum(0))
            g = dyf * hg.master
            dx = rstd[:, None] * (g - g.mean(-1, keepdim=True) - xhat * (g * xhat).mean(-1, keepdim=True))
            dx = dx.reshape(B, T, D)
        if hg.segs[0].trainable:
            hg.ready()
            hb.ready()
        return dx, None, None, None, None, None


def layer_norm(x: torch.Tensor, hg: Handle, hb: Handle, out_dtype=None) -> torch.Tensor:
    if x.dim() == 2:
        x = x.unsqueeze(0)
    out_dtype = out_dtype or hg.store.compute_dtype
    hg.note_use()
    hb.note_use()
    return _LayerNorm.apply(x, hg.param, hb.param, hg, hb, out_dtype)


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
        if _hip(x):
            out = _ext.load().residual_fwd(x, y2, hs.master if hs is not None else None, mask)
        else:
            r = y2.float().reshape(B, T, D)
            if hs is not None:
                r = r * hs.master
            if mask is not None:
                r = r * mask.view(B, 1, 1)
            out = x.float() + r
        ctx.save_for_backward(y2 if hs is not None else None, mask)
        ctx.hs = hs
        ctx.shape = (B, T, D)
        ctx.ydtype = y.dtype
        ctx.yshape = y.shape
        return out

    @staticmethod
    def backward(ctx, dout):
        y2, mask = ctx.saved_tensors
        hs = ctx.hs
        B, T, D = ctx.shape
        dout = dout.contiguous()
        if hs is None and mask is None:
            dy = dout.reshape(B * T, D).to(ctx.ydtype)
        elif _hip(dout):
            dy = _ext.load().residual_bwd(dout, y2, hs.master if hs is not None else None, mask,
                                          hs.grad if (hs is not None and hs.segs[0].trainable) else None,
                                          ctx.ydtype)
        else:
            d = dout.reshape(B, T, D)
            if mask is not None:
                d = d * mask.view(B, 1, 1)
            if hs is not None:
                if hs.segs[0].trainable:
                    hs.grad.add_((d * y2.float().reshape(B, T, D)).sum((0, 1)))
                d = d * hs.master
            dy = d.reshape(B * T, D).to(ctx.ydtype)
        if hs is not None and hs.segs[0].trainable:
            hs.ready()
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
        B, S, three_d = qkv.shape
        D = three_d // 3
        hd = D // heads
        if _hip(qkv):
            o, lse = _ext.load().attn_fwd(qkv, heads)
        else:
            q, k, v = qkv.float().view(B, S, 3, heads, hd).unbind(2)
            z = torch.einsum("bqhd,bkhd->bhqk", q / math.sqrt(hd), k)
            lse = torch.logsumexp(z, -1)
            p = torch.exp(z - lse[..., None])
            o = torch.einsum("bhqk,bkhd->bqhd", p, v).reshape(B, S, D).to(qkv.dtype)
        ctx.save_for_backward(qkv, o, lse)
        ctx.heads = heads
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        heads = ctx.heads
        B, S, three_d = qkv.shape
        D = three_d // 3
        hd = D // heads
        do = do.contiguous()
        if _hip(qkv):
            dqkv = _ext.load().attn_bwd(do, qkv, o, lse, heads)
        else:
            q, k, v = qkv.float().view(B, S, 3, heads, hd).unbind(2)
            dof = do.float().view(B, S, heads, hd)
            sc = 1.0 / math.sqrt(hd)
            z = torch.einsum("bqhd,bkhd->bhqk", q * sc, k)
            p = torch.exp(z - lse[..., None])
            dv = torch.einsum("bhqk,bqhd->bkhd", p, dof)
            dp = torch.einsum("bqhd,bkhd->bhqk", dof, v)
            delta = (dof * o.float().view(B, S, heads, hd)).sum(-1).permute(0, 2, 1)  # b h q
            ds = p * (dp - delta[..., None])
            dq = torch.einsum("bhqk,bkhd->bqhd", ds, k) * sc
            dk = torch.einsum("bhqk,bqhd->bkhd", ds, q) * sc
            dqkv = torch.stack([dq, dk, dv], 2).reshape(B, S, three_d).to(qkv.dtype)
        return dqkv, None


def attention(qkv: torch.Tensor, heads: int) -> torch.Tensor:
    return _Attention.apply(qkv, heads)
