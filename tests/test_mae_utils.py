"""Masking invariants, patchify, masked MSE, sincos table (reference utils_mae.py / utils.py)."""

import numpy as np
import torch

from jumbo_mae_tpu_amd.utils import mae as U
from jumbo_mae_tpu_amd.utils.posemb import fixed_sincos2d_embeddings


def test_masking_invariants_shared():
    noise = torch.rand(196)
    ids_shuffle, ids_restore, ids_keep, mask = U.masking_ids(noise, 49)
    assert torch.equal(ids_shuffle[ids_restore], torch.arange(196))
    assert mask.sum().item() == 196 - 49
    assert torch.all(mask[ids_keep] == 0)
    x = torch.randn(4, 196, 8)
    kept, m, restore = U.random_masking(x, None, 49, noise=noise)
    assert kept.shape == (4, 49, 8) and m.shape == (4, 196)
    assert torch.equal(kept, x[:, ids_shuffle[:49]])
    # one permutation shared by the whole batch (quirk Q1)
    assert torch.equal(m[0], m[3])


def test_masking_padding_mask():
    noise = torch.rand(16)
    x = torch.randn(2, 16, 3)
    pad = (torch.arange(16) < 11).float().expand(2, 16).clone()
    pad[1, 5:] = 0
    kept, m, restore, pad_kept = U.random_masking(x, None, 4, noise=noise, padding_mask=pad)
    ids = torch.argsort(noise)[:4]
    assert torch.equal(pad_kept, pad[:, ids]) and torch.equal(kept, x[:, ids])
    # per-sample ids gather per row
    noise2 = torch.rand(2, 16)
    *_, pad_kept2 = U.random_masking(x, None, 4, mode="per-sample", noise=noise2, padding_mask=pad)
    for b in range(2):
        assert torch.equal(pad_kept2[b], pad[b, torch.argsort(noise2[b])[:4]])


def test_masking_per_sample():
    noise = torch.rand(3, 16)
    x = torch.randn(3, 16, 2)
    kept, m, restore = U.random_masking(x, None, 4, mode="per-sample", noise=noise)
    assert kept.shape == (3, 4, 2)
    assert torch.all(m.sum(-1) == 12)
    for b in range(3):
        ids = torch.argsort(noise[b])[:4]
        assert torch.equal(kept[b], x[b, ids])


def test_patchify_roundtrip_and_order():
    img = torch.randn(2, 32, 48, 3)
    p = U.extract_patches(img, 16)
    assert p.shape == (2, 6, 768)
    # element order (ph, pw, c): patch (0,1), pixel (ph=2, pw=5, c=1)
    assert p[0, 1, (2 * 16 + 5) * 3 + 1] == img[0, 2, 16 + 5, 1]
    assert torch.equal(U.extract_patches_nchw(img.permute(0, 3, 1, 2), 16), p)
    sq = torch.randn(2, 32, 32, 3)
    assert torch.equal(U.merge_patches(U.extract_patches(sq, 16), 16), sq)


def test_patch_mse_loss_formula():
    out = torch.randn(3, 5, 4)
    tgt = torch.randn(3, 5, 4)
    valid = torch.tensor([[1, 0, 1, 0, 0], [1, 1, 1, 1, 1], [0, 0, 0, 0, 1.0]])
    ref = 0.0
    for b in range(3):
        errs = [((tgt[b, n] - out[b, n]) ** 2).mean() for n in range(5) if valid[b, n] > 0]
        ref += sum(errs) / len(errs)
    ref /= 3
    assert torch.allclose(U.patch_mse_loss(out, tgt, valid), torch.tensor(float(ref)), atol=1e-6)
    assert torch.allclose(U.patch_mse_loss(out, tgt), ((tgt - out) ** 2).mean(), atol=1e-6)


def test_mask_helpers():
    a, b = torch.tensor([1.0, 0, 1, 0]), torch.tensor([1.0, 1, 0, 0])
    assert torch.equal(U.mask_union(a, b), torch.tensor([1.0, 1, 1, 0]))
    assert torch.equal(U.mask_intersection(a, b), torch.tensor([1.0, 0, 0, 0]))
    assert torch.equal(U.mask_not(a), torch.tensor([0.0, 1, 0, 1]))
    x = torch.arange(4.0)
    assert torch.equal(U.mask_select(a, x), torch.tensor([0.0, 1, 0, 3]))


def test_sincos_table_values():
    t = fixed_sincos2d_embeddings(14, 14, 512).numpy()
    assert t.shape == (14, 14, 512)
    freqs = 1.0 / (10000.0 ** np.linspace(0, 1, 128))  # linspace WITH endpoint (reference quirk)
    # row y=3, col x=5: [sin(5 f), cos(5 f), sin(3 f), cos(3 f)]
    np.testing.assert_allclose(t[3, 5, :128], np.sin(5 * freqs), atol=1e-5)
    np.testing.assert_allclose(t[3, 5, 128:256], np.cos(5 * freqs), atol=1e-5)
    np.testing.assert_allclose(t[3, 5, 256:384], np.sin(3 * freqs), atol=1e-5)
    np.testing.assert_allclose(t[3, 5, 384:], np.cos(3 * freqs), atol=1e-5)
    assert abs(freqs[-1] - 1e-4) < 1e-12


def test_flop_counts_match_baseline():
    """Forward FLOPs/image of SURVEY.md §2.2 / BASELINE.md (20.7 GF ViT-B, 45.3 GF ViT-L) within 2%."""
    from jumbo_mae_tpu_amd.config import decoder_config, vit_config
    from jumbo_mae_tpu_amd.utils.flops import mfu, pretrain_fwd_flops_per_image
    for name, ref in (("vit_base_patch16", 20.7e9), ("vit_large_patch16", 45.3e9)):
        f = pretrain_fwd_flops_per_image(vit_config(name, labels=0, posemb="sincos2d"), decoder_config())
        assert abs(f - ref) / ref < 0.02, (name, f)
    assert abs(mfu(1000.0, 1e12, 2, peak=1e15) - 1.5) < 1e-9


def test_mixup_plan_matches_reference_mask_formulation():
    """CutMix box as pixel ranges == the reference's linspace-grid mask (utils.py:66-111), and
    the own-label weight is the kept-area fraction; Mixup blends with ratio."""
    import numpy as np

    from jumbo_mae_tpu_amd.utils.mixup import Mixup

    torch.manual_seed(0)
    imgs = torch.rand(6, 3, 32, 24)
    labels = torch.nn.functional.one_hot(torch.arange(6), 10).float()
    for seed in range(20):
        mx = Mixup(0.8, 1.0, seed=seed)
        plan = mx.plan(6, 32, 24, "cpu", torch.Generator().manual_seed(seed))
        out = Mixup.mix_images(imgs, plan)
        other = imgs[plan["perm"]]
        if plan["mode"] == "mixup":
            ref = plan["ratio"] * imgs + (1 - plan["ratio"]) * other
        else:
            rs = np.random.default_rng(seed)
            rs.uniform()  # mode draw
            ratio = float(rs.beta(1.0, 1.0))
            size = (1 - ratio) ** 0.5
            xs, ys = rs.uniform(size=2)
            xr, yr = torch.linspace(0, 1, 24), torch.linspace(0, 1, 32)
            xm = (xs - 0.5 * size <= xr) & (xr < xs + 0.5 * size)
            ym = (ys - 0.5 * size <= yr) & (yr < ys + 0.5 * size)
            keep = (~(ym[:, None] & xm[None, :])).float()
            ref = keep * imgs + (1 - keep) * other
            assert abs(plan["label_w"] - keep.mean().item()) < 1e-6
        assert torch.allclose(out, ref)
        lab = Mixup.mix_labels(labels, plan)
        assert torch.allclose(lab.sum(-1), torch.ones(6))
