"""Optimizer / schedule semantics vs per-leaf re-statements of the optax transformations."""

import math

import numpy as np
import pytest
import torch

from jumbo_mae_tpu_amd.config import DecoderConfig, ViTConfig
from jumbo_mae_tpu_amd.models.mae import PretrainModel
from jumbo_mae_tpu_amd.optim.flat import FlatOptimizer, layer_index
from jumbo_mae_tpu_amd.optim.schedule import warmup_cosine_decay_schedule


def test_schedule_boundaries():
    s = warmup_cosine_decay_schedule(1e-6, 1e-3, 10, 110, 1e-5)
    assert s(0) == pytest.approx(1e-6)
    assert s(5) == pytest.approx(1e-6 + 0.5 * (1e-3 - 1e-6))
    assert s(10) == pytest.approx(1e-3)
    alpha = 1e-5 / 1e-3
    # cosine over decay_steps - warmup = 100 steps (Q17)
    assert s(60) == pytest.approx(1e-3 * ((1 - alpha) * 0.5 * (1 + math.cos(math.pi * 0.5)) + alpha))
    assert s(110) == pytest.approx(1e-5)
    assert s(10_000) == pytest.approx(1e-5)
    z = warmup_cosine_decay_schedule(1e-6, 3.0, 0, 100, 1e-6)
    assert z(0) == pytest.approx(3.0)


def test_layer_index_labels():
    assert layer_index(("model", "layer_3", "attn", "wq", "kernel"), 12) == 4
    assert layer_index(("model", "embed", "wte", "kernel"), 12) == 0
    assert layer_index(("model", "cls_tokens"), 12) == 12
    assert layer_index(("model", "jumbo_mlp", "w1", "kernel"), 12) == 12
    assert layer_index(("decoder_model", "dec_layer_0", "ff"), 12) == 12


def _model():
    vc = ViTConfig(layers=2, dim=16, heads=2, labels=0, image_size=16, patch_size=8, posemb="learnable")
    dc = DecoderConfig(dec_layers=1, dec_dim=8, dec_heads=2, image_size=16, patch_size=8)
    return PretrainModel(vc, dc).to("cpu", seed=0)


def _leaves(store, flat):
    return {s.key: flat[s.offset:s.offset + s.numel].clone().double().view(s.shape) for s in store.segments}


def _ref_step(kind, p, g, st, count, lr, s, b1=0.9, b2=0.95, eps=1e-8, wd=0.05, clip=0.0, llrd=None,
              mom=0.9, tc=1e-3):
    """One optax update on dicts of leaves (float64)."""
    if clip > 0:
        gn = math.sqrt(sum(float((v ** 2).sum()) for v in g.values()))
        if gn >= clip:
            g = {k: v / gn * clip for k, v in g.items()}
    t = count + 1
    new = {}
    for k in p:
        kernel = k.endswith("/kernel")
        scale = llrd[k] if llrd else 1.0
        if kind in ("adamw", "lamb"):
            st["mu"][k] = b1 * st["mu"][k] + (1 - b1) * g[k]
            st["nu"][k] = b2 * st["nu"][k] + (1 - b2) * g[k] ** 2
            u = (st["mu"][k] / (1 - b1 ** t)) / (torch.sqrt(st["nu"][k] / (1 - b2 ** t)) + eps)
            if kernel:
                u = u + wd * p[k]
            if kind == "lamb" and kernel:
                pn, un = p[k].norm(), u.norm()
                if pn > 0 and un > 0:
                    u = u * (pn / un)
            new[k] = p[k] - lr * u * scale
        elif kind == "lars":
            u = g[k]
            pn, un = p[k].norm(), u.norm()
            tr = tc * pn / un if (pn > 0 and un > 0) else 1.0
            u = -lr * (u * tr)
            st["tr"][k] = u + mom * st["tr"][k]
            new[k] = p[k] + st["tr"][k] * scale
        else:
            st["tr"][k] = g[k] + mom * st["tr"][k]
            new[k] = p[k] - lr * st["tr"][k] * scale
    return new


@pytest.mark.parametrize("kind", ["adamw", "lamb", "lars", "sgd"])
@pytest.mark.parametrize("clip,lr_decay", [(0.0, 1.0), (0.3, 0.75)])
def test_flat_optimizer_matches_optax_semantics(kind, clip, lr_decay):
    m = _model()
    sched = warmup_cosine_decay_schedule(1e-6, 1e-2, 2, 8, 1e-5)
    opt = FlatOptimizer(m.store, kind, sched, b1=0.9, b2=0.95, eps=1e-8, weight_decay=0.05, lr_decay=lr_decay,
                        num_layers=2, clip_grad=clip)
    p = _leaves(m.store, m.store.master)
    st = {"mu": {k: torch.zeros_like(v) for k, v in p.items()}, "nu": {k: torch.zeros_like(v) for k, v in p.items()},
          "tr": {k: torch.zeros_like(v) for k, v in p.items()}}
    llrd = {s.key: (lr_decay ** (2 - layer_index(s.path, 2)) if lr_decay < 1 else 1.0) for s in m.store.segments}
    gen = torch.Generator().manual_seed(0)
    for c in range(4):
        m.store.grad.copy_(torch.randn(m.store.total, generator=gen) * 0.1)
        g = _leaves(m.store, m.store.grad)
        lr = opt.step()
        assert lr == pytest.approx(sched(c))
        wd = 0.05 if kind in ("adamw", "lamb") else 0.0
        p = _ref_step(kind, p, g, st, c, lr, None, wd=wd, clip=clip, llrd=llrd)
        ours = _leaves(m.store, m.store.master)
        for k in p:
            np.testing.assert_allclose(ours[k].numpy(), p[k].numpy(), rtol=2e-5, atol=3e-6, err_msg=k)


def test_optimizer_state_roundtrip():
    m = _model()
    opt = FlatOptimizer(m.store, "adamw", warmup_cosine_decay_schedule(1e-6, 1e-3, 2, 8, 1e-5))
    m.store.grad.normal_()
    opt.step()
    sd = opt.state_dict()
    opt2 = FlatOptimizer(m.store, "adamw", warmup_cosine_decay_schedule(1e-6, 1e-3, 2, 8, 1e-5))
    opt2.load_state_dict(sd)
    assert opt2.count == 1
    assert torch.equal(opt2.mu, opt.mu) and torch.equal(opt2.nu, opt.nu)


def test_optimizer_state_from_older_padding():
    """A sidecar written when the flat total was padded to 64 elements (round <= 3) resumes into
    today's TOTAL_ALIGN-padded buffers: the common prefix is copied, the padding tail zeroed."""
    m = _model()
    opt = FlatOptimizer(m.store, "adamw", warmup_cosine_decay_schedule(1e-6, 1e-3, 2, 8, 1e-5))
    m.store.grad.normal_()
    m.store.grad[m.store.used_numel():] = 0
    opt.step()
    sd = opt.state_dict()
    old_total = -(-m.store.used_numel() // 64) * 64
    assert old_total < m.store.total
    old = {k: (v[:old_total].clone() if isinstance(v, torch.Tensor) else v) for k, v in sd.items()}
    opt2 = FlatOptimizer(m.store, "adamw", warmup_cosine_decay_schedule(1e-6, 1e-3, 2, 8, 1e-5))
    opt2.mu.fill_(7.0)
    opt2.load_state_dict(old)
    assert torch.equal(opt2.mu, opt.mu) and torch.equal(opt2.nu, opt.nu)
    # a larger saved buffer (a store padded for more ranks) loads too while its tail is zero
    big = {k: (torch.cat([v, torch.zeros(128)]) if isinstance(v, torch.Tensor) else v) for k, v in sd.items()}
    opt2.load_state_dict(big)
    assert torch.equal(opt2.nu, opt.nu)
    bad = dict(big, mu=torch.cat([sd["mu"], torch.ones(128)]))
    with pytest.raises(ValueError):
        opt2.load_state_dict(bad)
    with pytest.raises(ValueError):
        opt2.load_state_dict(dict(sd, mu=sd["mu"][:m.store.used_numel() - 1]))
