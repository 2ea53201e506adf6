"""Fused transformer-block autograd Functions (one autograd node per layer).

A block's forward is a fixed chain of fused kernels and GEMMs; its backward is written out by
hand so that (i) the residual-stream gradient never goes through autograd's generic adds,
slice-backward zero fills or concat copies -- the passthrough add is fused into the LayerNorm
backward kernel and the CLS / patch halves of the Jumbo merge are read and written as strided
views in place; (ii) exactly the tensors the kernels need are saved; (iii) every parameter
gradient is accumulated straight into the flat fp32 buffer and the DP reducer is told as soon as
it is final.

JumboBlock = JumboLayer (/root/reference/src/modeling.py:169-206):
    x1 = x + dp1(s1 * Attn(LN1 x))
    c  = LN3(x1[:, :3].reshape(B, 3D));  c' = c + dp3(s3 * JumboMLP(c))     (shared MLP)
    p' = x1[:, 3:] + dp2(s2 * FF(LN2 x1[:, 3:]))
    x2 = concat(c'.reshape(B, 3, D), p')
ViTBlock = ViTLayer (modeling.py:150-167), the MAE decoder block.
"""

from __future__ import annotations


import torch

from typing import NamedTuple

from . import dropout as Dr
from . import prims as P


LINKS = True  # A/B switch (tools/ab_bench.py)
# forward hand-off of the upper block's LN1 (Link.ln1); A/B switch
FWD_LINKS = True


class Link:
    """Hand-off between two consecutive fused blocks (the model's layer loop creates one per
    boundary).  The lower block's forward publishes its patch-branch residual (y, s2, mask, bias,
    t0) as a ``P.ResSpec``; the upper block's backward fuses that residual's backward into its LN1
    backward -- whose dx IS the lower block's dx2 -- and leaves dy / bias_done here, so the lower
    block skips a pass that would re-read dx2 from HBM.

    Forward direction: when the layer loop names the upper block's LN1 (``ln1`` = (gamma, beta)
    handles), the lower block computes that LayerNorm in the same pass as its last residual add and
    leaves (h1, mean, rstd) here for the upper block, which would otherwise re-read x2 from HBM."""

    __slots__ = ("spec", "dy", "done", "dx_key", "ln1", "h1")

    def __init__(self, ln1=None):
        self.spec = None
        self.dy = None
        self.done = False
        self.dx_key = None
        self.ln1 = ln1
        self.h1 = None

    def put_h1(self, x2: torch.Tensor, h1, mu, rs):
        self.h1 = (x2.data_ptr(), tuple(x2.shape), h1, mu, rs)

    def take_h1(self, x: torch.Tensor):
        """(h1, mean, rstd) of LN1(x) if the lower block produced them for exactly this x."""
        if self.h1 is None:
            return None
        ptr, shape, h1, mu, rs = self.h1
        self.h1 = None
        if (ptr, shape) != (x.data_ptr(), tuple(x.shape)):
            return None
        return h1, mu, rs

    def take(self, dx2: torch.Tensor):
        """The fused dy if the upper block produced one for exactly this dx2, else None."""
        if self.dy is None:
            return None
        if self.dx_key != (dx2.data_ptr(), tuple(dx2.shape)):
            # the upper block already accumulated this residual's parameter gradients: falling
            # back to a second residual backward would count them twice
            raise RuntimeError("fused residual hand-off: dx2 is not the upper block's LN1 output")
        dy, done = self.dy, self.done
        self.dy = None
        return dy, done


class Drops(NamedTuple):
    """Dropout seeds of one fused block (reference modeling.py:133-148), drawn by the layer in the
    per-op path's order -- attention probabilities, attention output, (jumbo MLP hidden, output,)
    FF hidden, FF output -- so both paths apply the same masks.  Masks are regenerated from the
    seeds in the backward (csrc/common.h drop_keep): the attention probabilities inside the
    attention kernels, the FF hidden on the saved gelu(h) / gelu'(h) pair (the FF2 data-gradient
    epilogue then needs no mask), the Dense outputs on the branch output and its gradient."""
    rate: float
    attn: torch.Tensor
    wo: torch.Tensor
    fh: torch.Tensor
    fo: torch.Tensor
    jh: torch.Tensor | None = None
    jo: torch.Tensor | None = None


def _attn_fwd(attn, h1, B, S, dr: Drops | None = None):
    qkv = P.linear_fwd(h1, attn.qkv_k, attn.qkv_b)
    o, lse = P.attn_fwd(qkv.view(B, S, -1), attn.heads, drop=(dr.attn, dr.rate) if dr is not None else None)
    a = P.linear_fwd(o.view(B * S, -1), attn.wo_k, attn.wo_b)
    return qkv, o, lse, a


def _od(dr: Drops | None, name: str, base):
    """The residual kernels' descriptor of a Dense output's dropout: (seed, rate, branch tensor)."""
    return None if dr is None else (getattr(dr, name), dr.rate, base)


def _attn_bwd(attn, da, h1, qkv, o, lse, B, S, wo_bias_done=False, dr: Drops | None = None):
    do = P.linear_bwd(da, o.view(B * S, -1), attn.wo_k, attn.wo_b, bias_done=wo_bias_done)
    dqkv, bd = P.attn_bwd(do, qkv.view(B, S, -1), o, lse, attn.heads, attn.qkv_b,
                          drop=(dr.attn, dr.rate) if dr is not None else None)
    return P.linear_bwd(dqkv.view(B * S, -1), h1, attn.qkv_k, attn.qkv_b, bias_done=bd)


def _ff_fwd(ff, h, train=True, rate=0.0, sh=None, so=None):
    """(saved, gelu, y, deriv): ``saved`` is gelu'(pre) when ``deriv`` (fused MFMA forward), else pre.
    With the dropout seed ``sh`` the hidden gelu(h) and gelu'(h) are masked together (in the GEMM
    epilogue, or one pass after; saved is then always the masked gelu').  The output's dropout is
    applied by the residual kernels that read y (``_od``)."""
    pre, g, deriv, dropped = P.linear_gelu_fwd_saved(h, ff.w1.k, ff.w1.b, need_pre=train,
                                                     drop=(sh, rate) if sh is not None else None)
    if sh is not None and not dropped:  # (the fused gelu' forward drops inside its epilogue)
        g, pre = Dr.gelu_drop(pre, None, sh, rate)  # saved: the masked, scaled bf16 gelu'
        deriv = True
    y = P.linear_fwd(g, ff.w2.k, ff.w2.b)  # its dropout (seed so) is applied where y is consumed
    return pre, g, y, deriv


def _ff_bwd(ff, dy, h, pre, g, w2_bias_done=False, dx_add=None, deriv=False, rate=0.0):
    """``rate``: the hidden dropout rate the forward folded into uint8 gelu' codes (``pre``)."""
    hb1 = ff.w1.b if ff.w1.k.segs[0].trainable else None
    dpre, bias_done = P.linear_gelu_bwd(dy, g, pre, ff.w2.k, ff.w2.b, hb1, w2_bias_done, deriv, rate)
    return P.linear_bwd(dpre, h, ff.w1.k, ff.w1.b, bias_done=bias_done, dx_add=dx_add)


def _note_uses(*handles):
    for h in handles:
        if h is not None:
            h.note_use()


def _attn_handles(attn):
    return (attn.qkv_k, attn.qkv_b, attn.wo_k, attn.wo_b)


def _ff_handles(ff):
    return (ff.w1.k, ff.w1.b, ff.w2.k, ff.w2.b)


class JumboBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, layer, m1, m2, m3, link_in, link_out, train=True, dr=None):
        B, S, D = x.shape
        C = layer.C
        J = C * D
        dt = layer.norm1.g.store.compute_dtype
        h1, mu1, rs1 = _ln1_fwd(x, layer, link_in, dt)
        qkv, o, lse, a = _attn_fwd(layer.attn, h1, B, S, dr)
        # residual + LN2 of the patch rows in one pass
        x1, hp, mup, rsp = P.residual_ln_fwd(x, a, layer.scale1, m1, layer.norm2.g, layer.norm2.b, C,
                                             drop=_od(dr, "wo", a))
        # jumbo branch: LN3 on the concatenated CLS tokens, residual on the *normalized* value
        cls_in = x1[:, :C].reshape(B, 1, J)
        # fp32 hc for the residual and its compute-dtype copy for the jumbo MLP, one pass
        hc, muc, rsc, hcb = P.ln_fwd(cls_in, layer.norm3.g, layer.norm3.b, torch.float32, dt)
        rate = dr.rate if dr is not None else 0.0
        jpre, jg, jy, jd = _ff_fwd(layer.jumbo_mlp, hcb, train, rate, dr and dr.jh, dr and dr.jo)
        # patch branch
        pin = x1[:, C:]
        fpre, fg, fy, fd = _ff_fwd(layer.ff, hp, train, rate, dr and dr.fh, dr and dr.fo)
        x2 = torch.empty_like(x1)
        P.residual_fwd(hc.view(B, 1, J), jy, layer.scale3, m3, out=x2[:, :C].reshape(B, 1, J), drop=_od(dr, "jo", jy))
        nl = link_out.ln1 if link_out is not None else None
        if nl is not None:  # patch-row residual + the upper block's LN1 over all rows, one pass
            _, h1n, mun, rsn = P.residual_ln_fwd(x1, fy, layer.scale2, m2, nl[0], nl[1], 0, C, out=x2,
                                                 drop=_od(dr, "fo", fy))
            link_out.put_h1(x2, h1n, mun, rsn)
        else:
            P.residual_fwd(pin, fy, layer.scale2, m2, out=x2[:, C:], drop=_od(dr, "fo", fy))
        ctx.save_for_backward(x, mu1, rs1, h1, qkv, o, lse, a, x1, muc, rsc, hcb, jpre, jg, jy,
                              hp, mup, rsp, fpre, fg, fy, m1, m2, m3)
        ctx.layer = layer
        ctx.link_in, ctx.link_out = link_in, link_out
        ctx.gelu_deriv = (jd, fd)  # FF1 saved gelu'(h) instead of h (jumbo MLP, patch FF)
        ctx.gelu_rate = rate  # hidden dropout folded into uint8 gelu' codes (P.gd_decode)
        ctx.dr = dr
        if link_out is not None:
            link_out.spec = P.ResSpec(fy, layer.scale2, m2, layer.ff.w2.b, C, drop=_od(dr, "fo", fy))
        return x2

    @staticmethod
    def backward(ctx, dx2):
        with P.paired_wgrads():  # FF2 + FF1 and Wo + QKV weight gradients as grouped launches
            dx = _jumbo_bwd(ctx, dx2)
        return dx, None, None, None, None, None, None, None, None, None


def _jumbo_bwd(ctx, dx2):
    (x, mu1, rs1, h1, qkv, o, lse, a, x1, muc, rsc, hcb, jpre, jg, jy,
     hp, mup, rsp, fpre, fg, fy, m1, m2, m3) = ctx.saved_tensors
    layer = ctx.layer
    dr = ctx.dr
    B, S, D = x.shape
    C = layer.C
    J = C * D
    dt = h1.dtype
    dx2 = dx2.contiguous()
    dx1 = torch.empty_like(dx2)
    a3 = a.view(B, S, D)
    da = torch.empty_like(a)
    da3 = da.view(B, S, D)
    # ---- jumbo branch: d hc = dx2_cls + JumboMLP'(s3 * dp3 * dx2_cls); dx1_cls = LN3'(d hc)
    dcls = dx2[:, :C].reshape(B, 1, J)
    djy, bd = P.residual_bwd(dcls, jy, layer.scale3, m3, dt, layer.jumbo_mlp.w2.b, drop=_od(dr, "jo", jy))
    # d hc = dcls + JumboMLP'(...) in fp32, the add fused into the jumbo dgrad's split-K reduce
    dhc = _ff_bwd(layer.jumbo_mlp, djy, hcb, jpre, jg, bd, dx_add=dcls.reshape(B, J),
                  deriv=ctx.gelu_deriv[0], rate=ctx.gelu_rate)
    P.ln_bwd(dhc, x1[:, :C].reshape(B, 1, J), muc, rsc, layer.norm3.g, layer.norm3.b,
             out=dx1[:, :C].reshape(B, 1, J))
    # attention-residual backward of the CLS rows (the patch rows ride on LN2' below, which
    # also marks scale1 ready: it must come last)
    P.residual_bwd(dx1[:, :C], a3[:, :C], layer.scale1, m1, dt, layer.attn.wo_b, out=da3[:, :C], mark_ready=False,
                   drop=_od(dr, "wo", a))
    # ---- patch branch: dx1[:, C:] = dx2[:, C:] + LN2'(FF'(s2 * dp2 * dx2[:, C:]))
    fused = ctx.link_out.take(dx2) if ctx.link_out is not None else None
    if fused is not None:  # computed by the upper block's LN1 backward
        dfy, bd = fused
    else:
        dfy, bd = P.residual_bwd(dx2[:, C:], fy, layer.scale2, m2, dt, layer.ff.w2.b, drop=_od(dr, "fo", fy))
    dhp = _ff_bwd(layer.ff, dfy, hp, fpre, fg, bd, deriv=ctx.gelu_deriv[1], rate=ctx.gelu_rate)
    # ... and the attention-residual backward of those rows in the same pass
    _, _, bd = P.ln_bwd(dhp, x1[:, C:], mup, rsp, layer.norm2.g, layer.norm2.b, dres=dx2[:, C:],
                        out=dx1[:, C:],
                        res=P.ResSpec(a3[:, C:], layer.scale1, m1, layer.attn.wo_b, 0, da3[:, C:],
                                      drop=_od(dr, "wo", a)), h=hp)
    # ---- attention branch: dx = dx1 + LN1'(Attn'(s1 * dp1 * dx1))
    dh1 = _attn_bwd(layer.attn, da, h1, qkv, o, lse, B, S, bd, dr)
    return _ln1_bwd(ctx, dh1, x, mu1, rs1, layer, dx1, h1)


def _ln1_fwd(x, layer, link_in, dt):
    """LN1 of the block input, or the copy the lower block computed in its last residual pass."""
    pre = link_in.take_h1(x) if link_in is not None else None
    if pre is not None:
        return pre
    return P.ln_fwd(x, layer.norm1.g, layer.norm1.b, dt)


def _ln1_bwd(ctx, dh1, x, mu1, rs1, layer, dx1, h1=None):
    """dx = dx1 + LN1'(dh1) into dx1; with a lower fused block linked, its patch-branch residual
    backward rides on the same pass (Link).  ``h1``: LN1's bf16 output (x-hat rebuilt from it)."""
    li = ctx.link_in
    if li is None or li.spec is None:
        return P.ln_bwd(dh1, x, mu1, rs1, layer.norm1.g, layer.norm1.b, dres=dx1, out=dx1, h=h1)
    dx, li.dy, li.done = P.ln_bwd(dh1, x, mu1, rs1, layer.norm1.g, layer.norm1.b, dres=dx1, out=dx1, res=li.spec,
                                  h=h1)
    li.dx_key = (dx.data_ptr(), tuple(dx.shape))
    li.spec = None
    return dx


def jumbo_block(layer, x, m1=None, m2=None, m3=None, link_in: Link | None = None, link_out: Link | None = None,
                dr: Drops | None = None):
    _note_uses(layer.norm1.g, layer.norm1.b, layer.norm2.g, layer.norm2.b, layer.norm3.g, layer.norm3.b,
               layer.scale1, layer.scale2, layer.scale3, *_attn_handles(layer.attn), *_ff_handles(layer.ff),
               *_ff_handles(layer.jumbo_mlp))
    return JumboBlockFn.apply(x.contiguous(), layer.norm1.g.param, layer, m1, m2, m3, link_in, link_out,
                              torch.is_grad_enabled(), dr)


class ViTBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, layer, m1, m2, link_in, link_out, train=True, dr=None):
        B, S, D = x.shape
        dt = layer.norm1.g.store.compute_dtype
        h1, mu1, rs1 = _ln1_fwd(x, layer, link_in, dt)
        qkv, o, lse, a = _attn_fwd(layer.attn, h1, B, S, dr)
        x1, h2, mu2, rs2 = P.residual_ln_fwd(x, a, layer.scale1, m1, layer.norm2.g, layer.norm2.b, 0,
                                             drop=_od(dr, "wo", a))
        fpre, fg, fy, fd = _ff_fwd(layer.ff, h2, train, dr.rate if dr is not None else 0.0, dr and dr.fh,
                                   dr and dr.fo)
        nl = link_out.ln1 if link_out is not None else None
        if nl is not None:  # last residual + the upper block's LN1, one pass
            x2, h1n, mun, rsn = P.residual_ln_fwd(x1, fy, layer.scale2, m2, nl[0], nl[1], 0, drop=_od(dr, "fo", fy))
            link_out.put_h1(x2, h1n, mun, rsn)
        else:
            x2 = P.residual_fwd(x1, fy, layer.scale2, m2, drop=_od(dr, "fo", fy))
        ctx.save_for_backward(x, mu1, rs1, h1, qkv, o, lse, a, x1, mu2, rs2, h2, fpre, fg, fy, m1, m2)
        ctx.layer = layer
        ctx.link_in, ctx.link_out = link_in, link_out
        ctx.gelu_deriv = (False, fd)
        ctx.gelu_rate = dr.rate if dr is not None else 0.0
        ctx.dr = dr
        if link_out is not None:
            link_out.spec = P.ResSpec(fy, layer.scale2, m2, layer.ff.w2.b, 0, drop=_od(dr, "fo", fy))
        return x2

    @staticmethod
    def backward(ctx, dx2):
        with P.paired_wgrads():  # FF2 + FF1 and Wo + QKV weight gradients as grouped launches
            dx = _vit_bwd(ctx, dx2)
        return dx, None, None, None, None, None, None, None, None


def _vit_bwd(ctx, dx2):
    x, mu1, rs1, h1, qkv, o, lse, a, x1, mu2, rs2, h2, fpre, fg, fy, m1, m2 = ctx.saved_tensors
    layer = ctx.layer
    dr = ctx.dr
    B, S, D = x.shape
    dt = h1.dtype
    dx2 = dx2.contiguous()
    fused = ctx.link_out.take(dx2) if ctx.link_out is not None else None
    if fused is not None:  # computed by the upper block's LN1 backward
        dfy, bd = fused
    else:
        dfy, bd = P.residual_bwd(dx2, fy, layer.scale2, m2, dt, layer.ff.w2.b, drop=_od(dr, "fo", fy))
    dh2 = _ff_bwd(layer.ff, dfy, h2, fpre, fg, bd, deriv=ctx.gelu_deriv[1], rate=ctx.gelu_rate)
    # LN2' with the attention-residual backward of its dx fused in (never write autograd's dx2)
    dx1, da, bd = P.ln_bwd(dh2, x1, mu2, rs2, layer.norm2.g, layer.norm2.b, dres=dx2,
                           res=P.ResSpec(a, layer.scale1, m1, layer.attn.wo_b, drop=_od(dr, "wo", a)), h=h2)
    dh1 = _attn_bwd(layer.attn, da, h1, qkv, o, lse, B, S, bd, dr)
    return _ln1_bwd(ctx, dh1, x, mu1, rs1, layer, dx1, h1)


def vit_block(layer, x, m1=None, m2=None, link_in: Link | None = None, link_out: Link | None = None,
              dr: Drops | None = None):
    _note_uses(layer.norm1.g, layer.norm1.b, layer.norm2.g, layer.norm2.b, layer.scale1, layer.scale2,
               *_attn_handles(layer.attn), *_ff_handles(layer.ff))
    return ViTBlockFn.apply(x.contiguous(), layer.norm1.g.param, layer, m1, m2, link_in, link_out,
                            torch.is_grad_enabled(), dr)
