"""Cross-replica BatchNorm for the linear-probe head.

Reference: ``nn.BatchNorm(use_running_average=det, axis_name="batch")`` inside ``LinearCLS``
(/root/reference/src/modeling.py:216-217).  Flax semantics: batch statistics
are ``pmean`` of per-device ``mean(x)`` and ``mean(x^2)``, ``var = max(0, mean2 - mean^2)``
(biased), eps 1e-5, running stats updated with momentum 0.99 (``ra = m*ra + (1-m)*stat``).
One packed all-reduce of ``[sum x, sum x^2]`` (2*J floats) in forward and one of
``[sum g, sum g*xhat]`` in backward.
"""

from __future__ import annotations

import torch
import torch.distributed as dist

from ..models.params import Handle


def _world(group):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group)
    return 1


class _SyncBN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, sp, bp, hs: Handle, hb: Handle, eps: float, group, stats_out):
        n_local = x.shape[0]
        world = _world(group)
        packed = torch.cat([x.sum(0), (x * x).sum(0)]) / n_local
        if world > 1:
            dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=group)
            packed /= world
        mean, mean2 = packed.chunk(2)
        var = torch.clamp(mean2 - mean * mean, min=0.0)
        rstd = torch.rsqrt(var + eps)
        xhat = (x - mean) * rstd
        y = xhat * hs.master + hb.master
        ctx.save_for_backward(xhat, rstd)
        ctx.hs, ctx.hb, ctx.group, ctx.world, ctx.n = hs, hb, group, world, n_local
        stats_out.append((mean, var))
        return y

    @staticmethod
    def backward(ctx, dy):
        xhat, rstd = ctx.saved_tensors
        hs, hb = ctx.hs, ctx.hb
        if hs.segs[0].trainable:
            hs.grad.add_((dy * xhat).sum(0))
            hb.grad.add_(dy.sum(0))
            hs.ready()
            hb.ready()
        dx = None
        if ctx.needs_input_grad[0]:
            g = dy * hs.master
            packed = torch.cat([g.sum(0), (g * xhat).sum(0)])
            if ctx.world > 1:
                dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=ctx.group)
            n = ctx.n * ctx.world
            sg, sgx = packed.chunk(2)
            dx = rstd * (g - sg / n - xhat * sgx / n)
        return dx, None, None, None, None, None, None, None


@torch.no_grad()
def _update_running(running_mean, running_var, mean, var, momentum):
    running_mean.mul_(momentum).add_((1 - momentum) * mean)
    running_var.mul_(momentum).add_((1 - momentum) * var)


def sync_batch_norm(x: torch.Tensor, hs: Handle, hb: Handle, running_mean: torch.Tensor,
                    running_var: torch.Tensor, training: bool, momentum: float = 0.99, eps: float = 1e-5,
                    group=None) -> torch.Tensor:
    x = x.float()
    if not training:
        return (x - running_mean) * torch.rsqrt(running_var + eps) * hs.master + hb.master
    hs.note_use()
    hb.note_use()
    stats: list = []
    y = _SyncBN.apply(x, hs.param, hb.param, hs, hb, eps, group, stats)
    mean, var = stats[0]
    _update_running(running_mean, running_var, mean, var, momentum)
    return y
