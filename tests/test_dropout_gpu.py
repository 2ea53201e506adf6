"""HIP dropout kernels (csrc/dropout.hip) against the CPU mirror of the same hash mask, and
activation checkpointing with dropout on the GPU path."""

import pytest
import torch

from jumbo_mae_tpu_amd.ops import dropout as Dr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ext():
    from jumbo_mae_tpu_amd.ops import _ext
    return _ext.load(True)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rate", [0.1, 0.5])
def test_dropout_apply_matches_mirror(ext, dtype, rate):
    torch.manual_seed(0)
    x = torch.randn(3, 50, 96, device="cuda").to(dtype)
    seed = torch.tensor([0x1234_5678_9ABC], dtype=torch.int64, device="cuda")
    y = ext.dropout_apply(x, seed, rate)
    m = Dr.keep_mask(seed.cpu(), x.numel(), rate).view(x.shape).cuda()
    ref = torch.where(m, x.float() / (1 - rate), torch.zeros((), device="cuda"))
    assert torch.equal(y != 0, m & (x != 0))
    assert torch.allclose(y.float(), ref.to(dtype).float(), rtol=0, atol=0)


def test_softmax_dropout_matches_mirror(ext):
    torch.manual_seed(1)
    z = torch.randn(2, 4, 37, 37, device="cuda") * 3  # S not a multiple of 64 (lane tails)
    seed = torch.tensor([987654321], dtype=torch.int64, device="cuda")
    rate = 0.2
    p, pd = ext.softmax_dropout_fwd(z, seed, rate)
    m = Dr.keep_mask_rows(seed.cpu(), z.numel() // z.shape[-1], z.shape[-1], rate).view(z.shape).cuda()
    zr = z.double().requires_grad_(True)
    pr = torch.softmax(zr, -1)
    ref = torch.where(m, pr / (1 - rate), torch.zeros((), device="cuda", dtype=torch.float64))
    assert (p.double() - pr).abs().max() < 1e-6
    assert (pd.double() - ref).abs().max() < 1e-5
    w = torch.randn_like(z)
    (ref * w.double()).sum().backward()
    dz = ext.softmax_dropout_bwd(w, p, seed, rate)
    assert (dz.double() - zr.grad).abs().max() < 1e-5


@pytest.mark.parametrize("pair", [True, False])
def test_gelu_drop_matches_mirror(ext, pair):
    torch.manual_seed(0)
    h = (torch.randn(37, 96, device="cuda") * 2).bfloat16()
    seed = torch.tensor([424242], dtype=torch.int64, device="cuda")
    rate = 0.3
    x = h.float()
    t = torch.tanh(0.7978845608028654 * (x + 0.044715 * x ** 3))
    g = 0.5 * x * (1 + t)
    d = 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * x * x)
    m = Dr.keep_mask(seed.cpu(), h.numel(), rate).view(h.shape).cuda().float() / (1 - rate)
    if pair:
        gb, db = g.bfloat16(), d.bfloat16()
        go, do = ext.gelu_drop(gb, db, seed, rate)
        assert go.data_ptr() == gb.data_ptr()  # in place
        assert torch.equal(go, (g.bfloat16().float() * m).bfloat16())
        assert torch.equal(do, (d.bfloat16().float() * m).bfloat16())
    else:
        go, do = ext.gelu_drop(h, None, seed, rate)
        assert (go.float() - g * m).abs().max().item() < 2e-2 * (g * m).abs().max().item()
        assert (do.float() - d * m).abs().max().item() < 2e-2 * (d * m).abs().max().item()


def test_dropout_apply_inplace_matches_mirror(ext):
    x = torch.randn(40, 64, device="cuda").bfloat16()
    seed = torch.tensor([7], dtype=torch.int64, device="cuda")
    ref = ext.dropout_apply(x, seed, 0.25)
    ext.dropout_apply_(x, seed, 0.25)
    assert torch.equal(x, ref)


@pytest.mark.parametrize("per_op_ref", [True])
def test_fused_block_dropout_matches_per_op_gpu(monkeypatch, per_op_ref):
    """Finetune ViT with dropout 0.1 on the GPU: the fused blocks (dropout inside the attention
    kernels, the FF hidden pair and the Dense outputs) == the per-op graph with the same seeds,
    up to bf16 rounding."""
    from jumbo_mae_tpu_amd.config import ViTConfig
    from jumbo_mae_tpu_amd.models.classifier import FinetuneModel

    res = []
    for per_op in ("0", "1"):
        monkeypatch.setenv("JMAE_PER_OP", per_op)
        vc = ViTConfig(layers=2, dim=128, heads=2, labels=16, image_size=64, patch_size=16, posemb="sincos2d",
                       dropout=0.1)
        m = FinetuneModel(vc, label_smoothing=0.1).to("cuda", torch.bfloat16, seed=0)
        imgs = torch.randint(0, 256, (8, 3, 64, 64), dtype=torch.uint8,
                             generator=torch.Generator().manual_seed(2)).cuda()
        labels = torch.arange(8, device="cuda")
        m.store.zero_grad()
        out = m.forward(imgs, labels, rngs={"dropout": torch.Generator(device="cuda").manual_seed(3)}, det=False)
        out["loss"].backward()
        torch.cuda.synchronize()
        res.append((float(out["loss"]), m.store.grad.clone()))
    assert abs(res[0][0] - res[1][0]) < 2e-2 * abs(res[1][0])
    assert float((res[0][1] - res[1][1]).norm() / res[1][1].norm()) < 3e-2


def test_model_dropout_grad_ckpt_matches_plain():
    """Finetune ViT with dropout 0.1 / droppath 0.1 on the GPU: checkpointed recompute regenerates
    the hash masks from the restored generator, so gradients match the plain run."""
    from jumbo_mae_tpu_amd.config import ViTConfig
    from jumbo_mae_tpu_amd.models.classifier import FinetuneModel

    def run(ckpt):
        vc = ViTConfig(layers=2, dim=128, heads=2, labels=16, image_size=64, patch_size=16, posemb="sincos2d",
                       droppath=0.1, dropout=0.1, grad_ckpt=ckpt)
        m = FinetuneModel(vc, label_smoothing=0.1).to("cuda", torch.bfloat16, seed=0)
        imgs = torch.randint(0, 256, (4, 3, 64, 64), dtype=torch.uint8,
                             generator=torch.Generator().manual_seed(2)).cuda()
        labels = torch.tensor([0, 1, 2, 3], device="cuda")
        m.store.zero_grad()
        out = m.forward(imgs, labels, rngs={"dropout": torch.Generator(device="cuda").manual_seed(3)}, det=False)
        out["loss"].backward()
        torch.cuda.synchronize()
        return float(out["loss"]), m.store.grad.clone()

    l0, g0 = run(False)
    l1, g1 = run(True)
    assert l0 == l1
    assert float((g1 - g0).norm() / g0.norm()) < 1e-4  # float-atomic order only
