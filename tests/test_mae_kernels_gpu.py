"""Mask-first MAE glue kernels (csrc/mae.hip) vs plain PyTorch fp32 references (MI355X):
kept-patch gather from uint8, embed finish, decoder unshuffle fwd/bwd, per-patch MSE fwd/bwd."""

import pytest
import torch

from jumbo_mae_tpu_amd.ops import mae as mae_ops
from jumbo_mae_tpu_amd.utils.mae import extract_patches_nchw, index_sequence, masking_ids

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ext():
    from jumbo_mae_tpu_amd.ops import _ext
    return _ext.load(True)


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _images(B, H=224, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randint(0, 256, (B, 3, H, H), dtype=torch.uint8, device="cuda", generator=g)


def _ids(B, N, K, per_sample, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    noise = torch.rand((B, N) if per_sample else (N,), device="cuda", generator=g)
    return masking_ids(noise, K)


def _ref_patches(img, p):
    return extract_patches_nchw(mae_ops.normalize_images(img), p)


@pytest.mark.parametrize("per_sample", [False, True])
@pytest.mark.parametrize("p,H", [(16, 224), (8, 32)])
def test_gather_patches(ext, per_sample, p, H):
    B = 5
    N = (H // p) ** 2
    K = N // 4
    img = _images(B, H)
    _, _, keep, _ = _ids(B, N, K, per_sample)
    out = ext.gather_patches(img, keep.to(torch.int32).contiguous(), p)
    ref = index_sequence(_ref_patches(img, p), keep).reshape(B * K, -1)
    assert out.dtype == torch.bfloat16 and out.shape == ref.shape
    assert (out.float() - ref).abs().max().item() < 2e-2


@pytest.mark.parametrize("per_sample", [False, True])
@pytest.mark.parametrize("with_pos", [True, False])
def test_embed_finish(ext, per_sample, with_pos):
    B, N, K, C, D = 4, 196, 49, 3, 256
    torch.manual_seed(0)
    e = torch.randn(B * K, D, device="cuda").bfloat16()
    pos = torch.randn(N, D, device="cuda") if with_pos else None
    cls = torch.randn(1, C, D, device="cuda")
    _, _, keep, _ = _ids(B, N, K, per_sample)
    out = ext.embed_finish(e, pos, keep.to(torch.int32).contiguous(), cls, B)
    ev = e.float().view(B, K, D)
    if with_pos:
        ev = ev + (pos[keep] if keep.dim() == 1 else pos[keep])
    ref = torch.cat([cls.expand(B, C, D), ev], 1)
    assert (out - ref).abs().max().item() < 1e-6


@pytest.mark.parametrize("per_sample", [False, True])
@pytest.mark.parametrize("d", [512, 128])
def test_unshuffle(ext, per_sample, d):
    B, N, K, C = 6, 196, 49, 3
    torch.manual_seed(1)
    y = torch.randn(B, C + K, d, device="cuda").bfloat16()
    tok = torch.randn(d, device="cuda")
    pos = torch.randn(N, d, device="cuda")
    _, restore, _, _ = _ids(B, N, K, per_sample)
    out = ext.unshuffle_fwd(y, tok, restore.to(torch.int32).contiguous(), pos, C)
    yr = y.float().requires_grad_()
    tr = tok.clone().requires_grad_()
    ref = mae_ops.unshuffle(yr, tr, restore, pos, C)
    assert (out - ref).abs().max().item() < 1e-6
    dout = torch.randn_like(ref)
    dy, dtok_part = ext.unshuffle_bwd(dout, restore.to(torch.int32).contiguous(), C, K)
    ref.backward(dout)
    assert (dy.float() - yr.grad).abs().max().item() <= 2e-2 * yr.grad.abs().max().item()
    assert rel(dtok_part.sum(0), tr.grad) < 1e-5
    # the partials' column sums added in place by the strided HIP column sum (Handle.accumulate_grad_rows)
    g = torch.full_like(tok, 0.25)
    ext.colsum_add_f32(dtok_part, g)
    assert rel(g - 0.25, tr.grad) < 1e-5


@pytest.mark.parametrize("rows,ld,n", [(512, 3 * 1024 + 49 * 1024, 3 * 1024), (7, 100, 96), (2048, 4096, 4096)])
def test_colsum_add_f32_strided(ext, rows, ld, n):
    """g += x.sum(0) for a row-strided fp32 view (the CLS-row slice of dx)."""
    torch.manual_seed(0)
    buf = torch.randn(rows, ld, device="cuda")
    x = buf[:, :n]
    g = torch.randn(n, device="cuda")
    ref = g.double() + x.double().sum(0)
    ext.colsum_add_f32(x, g)
    assert (g.double() - ref).abs().max().item() < 1e-4 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("norm_pix", [False, True])
@pytest.mark.parametrize("p,H", [(16, 224), (8, 32)])
def test_patch_mse(ext, norm_pix, p, H):
    B = 3
    N = (H // p) ** 2
    img = _images(B, H, seed=3)
    torch.manual_seed(2)
    pred = torch.randn(B * N, 3 * p * p, device="cuda").bfloat16()
    mse = ext.patch_mse_fwd(pred, img, p, norm_pix)
    t = _ref_patches(img, p).reshape(B * N, -1)
    if norm_pix:
        t = mae_ops.norm_pix(t)
    pr = pred.float().requires_grad_()
    ref = (t - pr).square().mean(-1)
    assert rel(mse, ref) < 1e-5
    dmse = torch.randn(B * N, device="cuda")
    dmse[::3] = 0.0  # unmasked rows: zero gradient, skipped by the kernel
    dpred = ext.patch_mse_bwd(pred, img, dmse, p, norm_pix)
    ref.backward(dmse)
    assert rel(dpred, pr.grad) < 1e-2
    assert (dpred[::3].float() == 0).all()


@pytest.mark.parametrize("mask_mode", ["shared", "per-sample"])
@pytest.mark.parametrize("norm_pix", [False, True])
def test_pretrain_fused_glue_matches_torch_path(mask_mode, norm_pix, monkeypatch):
    """Loss and every gradient of a tiny pretrain model with the HIP glue vs the same model with
    the glue forced onto the torch composition (HIP blocks/GEMMs in both)."""
    from jumbo_mae_tpu_amd.config import DecoderConfig, ViTConfig
    from jumbo_mae_tpu_amd.models.mae import PretrainModel

    vc = ViTConfig(layers=2, dim=128, heads=2, labels=0, image_size=64, patch_size=16, posemb="sincos2d",
                   image_mask_ratio=0.75, layerscale=True)
    dc = DecoderConfig(dec_layers=1, dec_dim=64, dec_heads=2, image_size=64, patch_size=16)
    img = _images(8, 64, seed=5)
    noise = torch.rand((16,) if mask_mode == "shared" else (8, 16), device="cuda",
                       generator=torch.Generator(device="cuda").manual_seed(7))
    grads, losses = [], []
    for fused in (True, False):
        model = PretrainModel(vc, dc, norm_pix_loss=norm_pix, mask_mode=mask_mode).to("cuda", torch.bfloat16, seed=0)
        if not fused:  # glue ops only (ops/mae.py) onto the torch composition
            real = mae_ops._ext

            class _NoHip:
                load = staticmethod(real.load)

                @staticmethod
                def use_hip(t):
                    return False

            monkeypatch.setattr(mae_ops, "_ext", _NoHip)
        try:
            model.store.grad.zero_()
            loss = model(img, noise=noise)["loss"]
            loss.backward()
        finally:
            monkeypatch.undo()
        losses.append(loss.item())
        grads.append(model.store.grad.clone())
    assert abs(losses[0] - losses[1]) < 1e-3 * abs(losses[1])
    assert rel(grads[0], grads[1]) < 2e-2


@pytest.mark.parametrize("M,N,K", [(1000, 1536, 512), (4096, 4096, 1024)])
def test_gemm_gelu_only_epilogue(ext, M, N, K):
    """Inference epilogue (activation only) == the activation output of the training epilogue."""
    torch.manual_seed(3)
    x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()
    b = torch.randn(N, device="cuda") * 0.1
    pre, g = ext.gemm_nt(x, w, b, True)
    (g_only,) = ext.gemm_nt(x, w, b, True, True)
    assert torch.equal(g_only, g)


def test_pretrain_loss_same_with_and_without_grad():
    from jumbo_mae_tpu_amd.config import DecoderConfig, ViTConfig
    from jumbo_mae_tpu_amd.models.mae import PretrainModel

    vc = ViTConfig(layers=2, dim=256, heads=4, labels=0, image_size=224, patch_size=16, posemb="sincos2d",
                   image_mask_ratio=0.75)
    dc = DecoderConfig(dec_layers=2, dec_dim=128, dec_heads=4, image_size=224, patch_size=16)
    model = PretrainModel(vc, dc).to("cuda", torch.bfloat16, seed=0)
    img = _images(64, 224, seed=9)
    noise = torch.rand(196, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1))
    l1 = model(img, noise=noise)["loss"].item()
    with torch.no_grad():
        l2 = model(img, noise=noise)["loss"].item()
    assert l1 == l2


@pytest.mark.parametrize("mode", ["none", "mixup", "cutmix"])
def test_mix_patches(ext, mode):
    from jumbo_mae_tpu_amd.utils.mixup import Mixup

    B = 6
    img = _images(B, 224, seed=11)
    plan = None
    if mode != "none":
        for seed in range(50):  # find a plan of the requested kind
            plan = Mixup(0.8, 1.0, seed=seed).plan(B, 224, 224, "cuda", torch.Generator(device="cuda").manual_seed(0))
            if plan["mode"] == mode and (mode == "mixup" or plan["box"][1] > plan["box"][0]):
                break
    rows = mae_ops.mixed_patches(img, plan, 16, torch.bfloat16)
    if plan:
        ref = extract_patches_nchw(Mixup.mix_images(mae_ops.normalize_images(img), plan), 16)
    else:
        ref = _ref_patches(img, 16)
    assert (rows.float() - ref.reshape(rows.shape)).abs().max().item() < 2e-2


@pytest.mark.parametrize("n,rows,N,K,cols", [(24, 512, 1024, 256, None), (5, 96, 512, 768, (256, 512)),
                                            (3, 4096, 256, 512, None)])
def test_gemm_tn_wgrad_segmented(ext, n, rows, N, K, cols):
    """Batched weight gradient over per-layer blocks read in place == the concatenated GEMM."""
    torch.manual_seed(4)
    dys = [torch.randn(rows, N, device="cuda").bfloat16() for _ in range(n)]
    xs = [torch.randn(rows, K, device="cuda").bfloat16() for _ in range(n)]
    r0, r1 = cols if cols else (0, N)
    g = torch.randn(r1 - r0, K, device="cuda")
    ref = g.double() + torch.cat(dys)[:, r0:r1].double().t() @ torch.cat(xs).double()
    ext.gemm_tn_wgrad_seg([d[:, r0:r1] for d in dys], xs, g)
    assert rel(g, ref) < 1e-5


@pytest.mark.parametrize("R,N,K", [(1, 196, 49), (64, 196, 49), (3, 1024, 256), (2, 17, 0)])
def test_mask_ids_matches_torch(ext, R, N, K):
    """csrc/mae.hip mask_ids (stable ranks) == the torch argsort composition of random_masking
    (utils_mae.py:88-102), including duplicated noise values (ties broken by index)."""
    g = torch.Generator(device="cuda").manual_seed(5)
    noise = torch.rand((R, N), device="cuda", generator=g)
    noise[:, 1::7] = noise[:, 0:1]  # ties
    x = noise[0] if R == 1 else noise
    sh, rs, keep32, rs32, mask = ext.mask_ids(x.contiguous(), K)
    ref_sh = torch.argsort(x, dim=-1, stable=True)
    ref_rs = torch.argsort(ref_sh, dim=-1, stable=True)
    assert torch.equal(sh, ref_sh) and torch.equal(rs, ref_rs)
    assert torch.equal(keep32.long(), ref_sh[..., :K]) and torch.equal(rs32.long(), ref_rs)
    assert torch.equal(mask, (ref_rs >= K).float())
    # the model entry point returns the same ids and the int32 copies the gather kernels read
    s2, r2, k2, m2 = masking_ids(x, K)
    assert torch.equal(s2, ref_sh) and torch.equal(k2._i32, keep32) and torch.equal(r2._i32, rs32)
