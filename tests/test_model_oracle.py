"""Our model (flat store, fused-op autograd, mask-first) vs the literal fp64 transcription of the
reference forward (models/oracle.py): loss and every gradient leaf of the Flax tree."""

import numpy as np
import pytest
import torch

from jumbo_mae_tpu_amd.config import DecoderConfig, ViTConfig
from jumbo_mae_tpu_amd.models import oracle
from jumbo_mae_tpu_amd.models.classifier import FinetuneModel
from jumbo_mae_tpu_amd.models.mae import PretrainModel


def _grads_match(store, tp, atol_scale=2e-4):
    flat = oracle.flatten(tp)
    total = np.sqrt(sum(float((v.grad.numpy() ** 2).sum()) for v in flat.values() if v.grad is not None))
    for s in store.segments:
        g = s.to_flax(store.grad[s.offset:s.offset + s.numel].numpy().reshape(s.shape))
        r = flat[s.key].grad
        r = np.zeros_like(g) if r is None else r.numpy()
        err = np.abs(g - r).max()
        assert err <= atol_scale * total + 1e-4 * np.abs(r).max(), (s.key, err, np.abs(r).max())


@pytest.mark.parametrize("layerscale,posemb,norm_pix,mode", [
    (False, "sincos2d", False, "shared"),
    (True, "sincos2d", True, "shared"),
    (True, "learnable", False, "per-sample"),
])
def test_pretrain_matches_oracle(layerscale, posemb, norm_pix, mode):
    torch.manual_seed(0)
    vc = ViTConfig(layers=2, dim=32, heads=4, labels=0, image_size=32, patch_size=8, posemb=posemb,
                   layerscale=layerscale, image_mask_ratio=0.75)
    dc = DecoderConfig(dec_layers=2, dec_dim=16, dec_heads=2, image_size=32, patch_size=8, dec_layerscale=layerscale)
    m = PretrainModel(vc, dc, norm_pix_loss=norm_pix, mask_mode=mode).to("cpu")
    m.store.master.add_(torch.randn_like(m.store.master) * 0.05)
    imgs = torch.randint(0, 256, (3, 3, 32, 32), dtype=torch.uint8)
    noise = torch.rand(16) if mode == "shared" else torch.rand(3, 16)
    out = m(imgs, noise=noise)
    out["loss"].backward()
    tp = oracle.tree_to_torch(m.flax_params())
    ref = oracle.mae_loss(tp, imgs, noise.double(), layers=2, dim=32, heads=4, dec_layers=2, dec_dim=16,
                          dec_heads=2, patch=8, mask_ratio=0.75, norm_pix_loss=norm_pix, posemb=posemb)
    ref.backward()
    assert abs(out["loss"].item() - ref.item()) < 1e-5 * max(1.0, abs(ref.item()))
    _grads_match(m.store, tp)


def test_param_count_vit_b_and_l():
    """Parameter totals of SURVEY.md §2.2 (ViT-B 154,191,360 / ViT-L 404,901,632 pretrain)."""
    from jumbo_mae_tpu_amd.config import decoder_config, vit_config
    for name, expect in (("vit_base_patch16", 154_191_360), ("vit_large_patch16", 404_901_632)):
        m = PretrainModel(vit_config(name, labels=0, posemb="sincos2d"), decoder_config())
        assert m.store.num_params() == expect


@pytest.mark.parametrize("batch_norm", [False, True])
def test_finetune_logits_match_oracle(batch_norm):
    torch.manual_seed(0)
    vc = ViTConfig(layers=2, dim=32, heads=4, labels=7, image_size=32, patch_size=8, posemb="learnable",
                   image_mask_ratio=None, batch_norm=batch_norm, linear_probing=batch_norm)
    m = FinetuneModel(vc).to("cpu")
    m.store.master.add_(torch.randn_like(m.store.master) * 0.05)
    imgs = torch.randint(0, 256, (5, 3, 32, 32), dtype=torch.uint8)
    logits, _ = m.logits(imgs, None, None, det=False)
    tp = oracle.tree_to_torch(m.flax_params(), requires_grad=False)
    x = oracle.normalize_nhwc(imgs)
    ref = oracle.classifier_logits(tp, x, layers=2, dim=32, heads=4, patch=8, posemb="learnable", training=True)
    assert torch.allclose(logits.double(), ref, atol=2e-5)
    if batch_norm:  # running stats updated with momentum 0.99 from the batch stats
        assert not torch.allclose(m.head.running_var, torch.ones_like(m.head.running_var))


def test_finetune_grads_match_oracle():
    torch.manual_seed(1)
    vc = ViTConfig(layers=1, dim=32, heads=2, labels=5, image_size=16, patch_size=8, posemb="learnable",
                   image_mask_ratio=None, layerscale=True)
    m = FinetuneModel(vc, label_smoothing=0.1).to("cpu")
    m.store.master.add_(torch.randn_like(m.store.master) * 0.05)
    imgs = torch.randint(0, 256, (4, 3, 16, 16), dtype=torch.uint8)
    labels = torch.tensor([0, 3, 1, 4])
    out = m(imgs, labels, rngs={}, det=False)
    out["loss"].backward()
    tp = oracle.tree_to_torch(m.flax_params())
    lg = oracle.classifier_logits(tp, oracle.normalize_nhwc(imgs), layers=1, dim=32, heads=2, patch=8)
    onehot = torch.nn.functional.one_hot(labels, 5).double() * 0.9 + 0.1 / 5
    ref = -(onehot * torch.log_softmax(lg, -1)).sum(-1).mean()
    ref.backward()
    assert abs(out["loss"].item() - ref.item()) < 1e-5
    _grads_match(m.store, tp)


def test_fused_blocks_match_per_op_with_droppath(monkeypatch):
    """The hand-written block backward (ops/blocks.py) == autograd over the per-op graph,
    with droppath + layerscale active (same RNG draws -> same masks)."""
    from jumbo_mae_tpu_amd.utils.rng import RngStreams
    vc = ViTConfig(layers=2, dim=32, heads=4, labels=0, image_size=32, patch_size=8, posemb="sincos2d",
                   layerscale=True, droppath=0.3)
    dc = DecoderConfig(dec_layers=2, dec_dim=16, dec_heads=2, image_size=32, patch_size=8, dec_layerscale=True,
                       dec_droppath=0.3)
    imgs = torch.randint(0, 256, (4, 3, 32, 32), dtype=torch.uint8)
    noise = torch.rand(16)
    res = []
    for per_op in ("0", "1"):
        monkeypatch.setenv("JMAE_PER_OP", per_op)
        m = PretrainModel(vc, dc).to("cpu", seed=0)
        with torch.no_grad():
            m.store.master.add_(torch.linspace(-0.02, 0.02, m.store.total))
        rng = RngStreams({"dropout": 5}, 0, "cpu").as_dict()
        loss = m(imgs, rngs=rng, noise=noise)["loss"]
        loss.backward()
        res.append((loss.item(), m.store.grad.clone()))
    assert abs(res[0][0] - res[1][0]) < 1e-6
    assert torch.allclose(res[0][1], res[1][1], atol=1e-6, rtol=1e-4)


@pytest.mark.parametrize("rate", [0.1, 0.5])
def test_fused_blocks_match_per_op_with_dropout(monkeypatch, rate):
    """Dropout > 0 on the fused blocks (attention probabilities, attention / FF / jumbo-MLP outputs
    and hidden layers; ops/blocks.py Drops) == the per-op graph with the same seeds: the layer draws
    them in the per-op order and every site uses the shared hash-mask convention."""
    from jumbo_mae_tpu_amd.utils.rng import RngStreams
    vc = ViTConfig(layers=2, dim=32, heads=4, labels=0, image_size=32, patch_size=8, posemb="sincos2d",
                   layerscale=True, droppath=0.2, dropout=rate)
    dc = DecoderConfig(dec_layers=2, dec_dim=16, dec_heads=2, image_size=32, patch_size=8, dec_layerscale=True,
                       dec_dropout=rate)
    imgs = torch.randint(0, 256, (4, 3, 32, 32), dtype=torch.uint8)
    noise = torch.rand(16)
    res = []
    for per_op in ("0", "1"):
        monkeypatch.setenv("JMAE_PER_OP", per_op)
        m = PretrainModel(vc, dc).to("cpu", seed=0)
        with torch.no_grad():
            m.store.master.add_(torch.linspace(-0.02, 0.02, m.store.total))
        rng = RngStreams({"dropout": 5}, 0, "cpu").as_dict()
        loss = m(imgs, rngs=rng, noise=noise)["loss"]
        loss.backward()
        res.append((loss.item(), m.store.grad.clone()))
    assert abs(res[0][0] - res[1][0]) < 1e-5 * max(1.0, abs(res[1][0]))
    assert torch.allclose(res[0][1], res[1][1], atol=1e-6, rtol=1e-4)
    # and the dropout is live: a different rate gives a different loss
    assert res[0][1].abs().sum() > 0


def test_forward_links_fuse_upper_ln1(monkeypatch):
    """Forward Link hand-off: each lower block computes the upper block's LN1 in its last residual
    pass (ops/blocks.py Link.ln1) -- fewer standalone LayerNorms, identical loss and gradients."""
    from jumbo_mae_tpu_amd.ops import blocks
    from jumbo_mae_tpu_amd.utils.rng import RngStreams
    vc = ViTConfig(layers=3, dim=32, heads=4, labels=0, image_size=32, patch_size=8, posemb="sincos2d",
                   layerscale=True, droppath=0.2)
    dc = DecoderConfig(dec_layers=3, dec_dim=16, dec_heads=2, image_size=32, patch_size=8, dec_layerscale=True)
    imgs = torch.randint(0, 256, (4, 3, 32, 32), dtype=torch.uint8)
    noise = torch.rand(16)
    calls = {"hits": 0}
    real = blocks.Link.take_h1

    def counting(self, x):
        out = real(self, x)
        calls["hits"] += out is not None
        return out

    monkeypatch.setattr(blocks.Link, "take_h1", counting)
    res = []
    for fwd in (False, True):
        monkeypatch.setattr(blocks, "FWD_LINKS", fwd)
        calls["hits"] = 0
        m = PretrainModel(vc, dc).to("cpu", seed=0)
        with torch.no_grad():
            m.store.master.add_(torch.linspace(-0.02, 0.02, m.store.total))
        rng = RngStreams({"dropout": 5}, 0, "cpu").as_dict()
        loss = m(imgs, rngs=rng, noise=noise)["loss"]
        loss.backward()
        res.append((loss.item(), m.store.grad.clone(), calls["hits"]))
    assert (res[0][2], res[1][2]) == (0, 4)  # 2 encoder + 2 decoder upper-block LN1s handed over
    assert abs(res[0][0] - res[1][0]) < 1e-6
    assert torch.allclose(res[0][1], res[1][1], atol=1e-6, rtol=1e-4)
