"""Route autograd gradients of directly-used parameter tensors into the flat grad buffer."""

from __future__ import annotations

import torch

from ..models.params import Handle


class _ParamValue(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p, h: Handle, dtype):
        ctx.h = h
        return h.master.to(dtype) if dtype != torch.float32 else h.master.clone()

    @staticmethod
    def backward(ctx, g):
        h = ctx.h
        if h.segs[0].trainable:
            h.accumulate_grad(g)
        return None, None, None


def param_value(h: Handle, dtype=torch.float32) -> torch.Tensor:
    """The fp32 master value of ``h`` as a differentiable tensor whose gradient lands in
    ``h.grad`` (used for cls tokens, learnable posemb, the MAE mask token)."""
    h.note_use()
    return _ParamValue.apply(h.param, h, dtype)
