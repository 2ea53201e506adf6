"""Hash-mask dropout (ops/dropout.py, csrc/dropout.hip): CPU mirror semantics here, HIP kernels
against that mirror in test_kernels_gpu.py::test_dropout_*."""

import torch

from jumbo_mae_tpu_amd.ops import dropout as Dr


def test_keep_mask_rate_and_determinism():
    seed = torch.tensor([123456789012345], dtype=torch.int64)
    m = Dr.keep_mask(seed, 200000, 0.3)
    assert abs(m.float().mean().item() - 0.7) < 0.005
    assert torch.equal(m, Dr.keep_mask(seed, 200000, 0.3))
    other = Dr.keep_mask(torch.tensor([987654321], dtype=torch.int64), 200000, 0.3)
    assert (m != other).float().mean().item() > 0.3  # independent streams per seed
    # neighbouring elements are not correlated
    f = m.float()
    c = ((f[1:] - f.mean()) * (f[:-1] - f.mean())).mean() / f.var()
    assert abs(c.item()) < 0.01


def test_mul32_matches_uint32_arithmetic():
    import numpy as np
    a = torch.randint(0, 2 ** 32, (1000,), dtype=torch.int64)
    for c in (0x85EBCA6B, 0xC2B2AE35, 1, 0xFFFFFFFF):
        ref = (a.numpy().astype(np.uint64) * np.uint64(c)) & np.uint64(0xFFFFFFFF)
        assert np.array_equal(Dr._mul32(a, c).numpy().astype(np.uint64), ref)


def test_dropout_backward_uses_the_forward_mask():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(4, 16, 24, requires_grad=True)
    y = Dr.dropout(x, 0.25, g)
    kept = y != 0
    assert abs(kept.float().mean().item() - 0.75) < 0.05
    assert torch.allclose(y[kept], x[kept] / 0.75)
    y.backward(torch.ones_like(y))
    assert torch.equal(x.grad != 0, kept)
    assert torch.allclose(x.grad[kept], torch.full_like(x.grad[kept], 1 / 0.75))


def test_softmax_dropout_grad_matches_autograd():
    g = torch.Generator().manual_seed(1)
    z = torch.randn(2, 3, 7, 9, dtype=torch.float64)
    state = g.get_state()
    zz = z.clone().requires_grad_(True)
    out = Dr.softmax_dropout(zz.float(), 0.2, g)
    w = torch.randn_like(out)
    (out * w).sum().backward()
    # reference: same seed -> same mask, plain torch autograd
    g2 = torch.Generator()
    g2.set_state(state)
    seed = Dr.draw_seed(g2, "cpu")
    m = Dr.keep_mask_rows(seed, z.numel() // z.shape[-1], z.shape[-1], 0.2).view(z.shape)
    zr = z.clone().float().requires_grad_(True)
    ref = torch.where(m, torch.softmax(zr, -1) / 0.8, torch.zeros(()))
    assert torch.allclose(out, ref, atol=1e-6)
    (ref * w).sum().backward()
    assert torch.allclose(zz.grad.float(), zr.grad, atol=1e-5)


def test_rate_edges():
    x = torch.randn(8, 8)
    assert Dr.dropout(x, 0.0, None) is x
    assert torch.count_nonzero(Dr.dropout(x, 1.0, None)) == 0


def test_dropout_seed_pool_one_draw_per_stack(monkeypatch):
    """models/vit.py dropout_seed_pool: the whole stack's seeds (and the input dropout's) come from
    ONE draw, sliced per layer in call order; layers without dropout get None."""
    from types import SimpleNamespace

    from jumbo_mae_tpu_amd.models import vit

    calls = []
    real = Dr.draw_seeds

    def counting(rng, device, n):
        calls.append(n)
        return real(rng, device, n)

    monkeypatch.setattr(Dr, "draw_seeds", counting)
    layers = [SimpleNamespace(dropout_rate=0.1, n_seeds=6), SimpleNamespace(dropout_rate=0.0, n_seeds=6),
              SimpleNamespace(dropout_rate=0.1, n_seeds=4)]
    g = torch.Generator().manual_seed(0)
    x = torch.randn(4, 8)
    y, seeds = vit.dropout_seed_pool(layers, g, "cpu", False, head=(x, 0.25))
    assert calls == [11]
    assert [None if s is None else len(s) for s in seeds] == [6, None, 4]
    assert len({int(t.item()) for s in seeds if s is not None for t in s}) == 10
    assert ((y == 0) | torch.isclose(y, x / 0.75)).all()
    calls.clear()
    y2, seeds2 = vit.dropout_seed_pool(layers, g, "cpu", True, head=(x, 0.25))  # eval: nothing drawn
    assert calls == [] and seeds2 == [None] * 3 and y2 is x
