"""End-to-end numerics of the HIP path (bf16 + fused kernels) against the fp32 CPU path."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


@pytest.mark.parametrize("layerscale", [False, True])
def test_pretrain_gpu_matches_cpu(layerscale):
    from jumbo_mae_tpu_amd.config import DecoderConfig, ViTConfig
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    vc = ViTConfig(layers=2, dim=128, heads=2, labels=0, image_size=64, patch_size=16, posemb="sincos2d",
                   layerscale=layerscale)
    dc = DecoderConfig(dec_layers=2, dec_dim=64, dec_heads=2, image_size=64, patch_size=16,
                       dec_layerscale=layerscale)
    cpu = PretrainModel(vc, dc).to("cpu", torch.float32, seed=0)
    gpu = PretrainModel(vc, dc).to("cuda", torch.bfloat16, seed=0)
    gpu.store.master.copy_(cpu.store.master)
    gpu.store.sync_shadow()
    imgs = torch.randint(0, 256, (8, 3, 64, 64), dtype=torch.uint8)
    noise = torch.rand(16)
    lc = cpu(imgs, noise=noise)["loss"]
    lc.backward()
    lg = gpu(imgs.cuda(), noise=noise.cuda())["loss"]
    lg.backward()
    torch.cuda.synchronize()
    assert abs(lc.item() - lg.item()) / lc.item() < 2e-2
    gc, gg = cpu.store.grad, gpu.store.grad.cpu()
    assert _cos(gc, gg) > 0.99
    for s in cpu.store.segments:
        a = gc[s.offset:s.offset + s.numel]
        b = gg[s.offset:s.offset + s.numel]
        if a.norm() > 1e-3 * gc.norm() / len(cpu.store.segments) ** 0.5:
            assert _cos(a, b) > 0.95, s.key


def test_pretrain_vit_large_step_runs():
    """One full ViT-L/16 step at a small batch: shapes of the headline config exercise every kernel."""
    from jumbo_mae_tpu_amd.config import decoder_config, vit_config
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.optim.flat import FlatOptimizer
    from jumbo_mae_tpu_amd.optim.schedule import warmup_cosine_decay_schedule
    from jumbo_mae_tpu_amd.train.engine import Trainer
    from jumbo_mae_tpu_amd.utils.rng import RngStreams
    vc = vit_config("vit_large_patch16", labels=0, posemb="sincos2d")
    m = PretrainModel(vc, decoder_config()).to("cuda", torch.bfloat16, seed=0)
    opt = FlatOptimizer(m.store, "adamw", warmup_cosine_decay_schedule(1e-6, 1e-3, 2, 10, 1e-5), b2=0.95,
                        weight_decay=0.05, num_layers=vc.layers)
    tr = Trainer(m, opt, None, RngStreams({}, 0, "cuda"))
    imgs = torch.randint(0, 256, (8, 3, 224, 224), dtype=torch.uint8, device="cuda")
    losses = [tr.train_step([(imgs,)])["loss"].item() for _ in range(4)]
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < losses[0]


@pytest.mark.parametrize("heads", [2, 4])
def test_finetune_long_sequence_gpu_matches_cpu(heads):
    """Classifier at 403 tokens (400 patches + 3 CLS > the 224-token fused attention limit): the
    blocks run the tile-streamed attention kernels and take the QKV bias gradient themselves.
    bf16 HIP loss / gradients against the fp32 CPU path (head dims 64 and 32)."""
    from jumbo_mae_tpu_amd.config import ViTConfig
    from jumbo_mae_tpu_amd.models.classifier import FinetuneModel
    vc = ViTConfig(layers=2, dim=128, heads=heads, labels=10, image_size=160, patch_size=8, posemb="learnable")
    assert (160 // 8) ** 2 + 3 > 224
    cpu = FinetuneModel(vc).to("cpu", torch.float32, seed=0)
    gpu = FinetuneModel(vc).to("cuda", torch.bfloat16, seed=0)
    gpu.store.master.copy_(cpu.store.master)
    gpu.store.sync_shadow()
    g = torch.Generator().manual_seed(0)
    imgs = torch.randint(0, 256, (4, 3, 160, 160), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (4,), generator=g)
    lc = cpu(imgs, labels)["loss"]
    lc.backward()
    lg = gpu(imgs.cuda(), labels.cuda())["loss"]
    lg.backward()
    torch.cuda.synchronize()
    assert abs(lc.item() - lg.item()) / lc.item() < 2e-2
    gc, gg = cpu.store.grad, gpu.store.grad.cpu()
    assert _cos(gc, gg) > 0.99
    for s in cpu.store.segments:
        a = gc[s.offset:s.offset + s.numel]
        b = gg[s.offset:s.offset + s.numel]
        if a.norm() > 1e-3 * gc.norm() / len(cpu.store.segments) ** 0.5:
            assert _cos(a, b) > 0.95, s.key


def _compare_leaves(cpu, gpu, lc, lg, strict=0.99, loose=0.95):
    """Loss within 2 %; flat-gradient cosine > 0.99; every 2-D (GEMM weight) leaf > ``strict``, the
    other leaves > ``loose`` (tiny gradients -- below 1e-3 of the per-leaf RMS norm -- are skipped)."""
    assert abs(lc.item() - lg.item()) / abs(lc.item()) < 2e-2, (lc.item(), lg.item())
    gc, gg = cpu.store.grad, gpu.store.grad.cpu()
    assert _cos(gc, gg) > 0.99
    bad = []
    for s in cpu.store.segments:
        a = gc[s.offset:s.offset + s.numel]
        b = gg[s.offset:s.offset + s.numel]
        if a.norm() <= 1e-3 * gc.norm() / len(cpu.store.segments) ** 0.5:
            continue
        c = _cos(a, b)
        if c < (strict if len(s.shape) == 2 else loose):
            bad.append((s.key, len(s.shape), round(c, 4)))
    assert not bad, bad


def test_pretrain_production_routing_matches_cpu():
    """ViT-B-width Jumbo MAE (dim 768, 224 px, batch 96) so that every Dense takes the production
    route: encoder rows 96 x 52 = 4992, patch-FF rows 4704 and decoder rows 96 x 199 >= 4096 run the
    hand-written MFMA GEMMs (FF1 saving gelu', FF2 data gradient x gelu' (DMUL), data gradients on
    the transposed weight shadows, TN weight gradients split over M, the deferred segmented jumbo
    weight gradient over both layers' CLS rows).  bf16 HIP step vs the fp32 CPU step
    (/root/reference/src/pretraining.py:87-122)."""
    from jumbo_mae_tpu_amd.config import DecoderConfig, ViTConfig
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    vc = ViTConfig(layers=2, dim=768, heads=12, labels=0, image_size=224, patch_size=16, posemb="sincos2d",
                   layerscale=True)
    dc = DecoderConfig(dec_layers=2, dec_dim=512, dec_heads=16, image_size=224, patch_size=16, dec_layerscale=True)
    cpu = PretrainModel(vc, dc).to("cpu", torch.float32, seed=0)
    gpu = PretrainModel(vc, dc).to("cuda", torch.bfloat16, seed=0)
    gpu.store.master.copy_(cpu.store.master)
    gpu.store.sync_shadow()
    g = torch.Generator().manual_seed(0)
    imgs = torch.randint(0, 256, (96, 3, 224, 224), dtype=torch.uint8, generator=g)
    noise = torch.rand(196, generator=g)
    lc = cpu(imgs, noise=noise)["loss"]
    lc.backward()
    lg = gpu(imgs.cuda(), noise=noise.cuda())["loss"]
    lg.backward()
    torch.cuda.synchronize()
    _compare_leaves(cpu, gpu, lc, lg)


def test_finetune_production_routing_matches_cpu():
    """Classifier at batch 32 x 199 tokens = 6368 encoder rows (>= 4096: MFMA GEMMs for every
    Dense but the 32-row jumbo MLP and the head), dim 768; bf16 HIP vs fp32 CPU
    (/root/reference/src/finetuning.py:84-106)."""
    from jumbo_mae_tpu_amd.config import ViTConfig
    from jumbo_mae_tpu_amd.models.classifier import FinetuneModel
    vc = ViTConfig(layers=2, dim=768, heads=12, labels=1000, image_size=224, patch_size=16, posemb="learnable",
                   layerscale=True)
    cpu = FinetuneModel(vc).to("cpu", torch.float32, seed=0)
    gpu = FinetuneModel(vc).to("cuda", torch.bfloat16, seed=0)
    gpu.store.master.copy_(cpu.store.master)
    gpu.store.sync_shadow()
    g = torch.Generator().manual_seed(0)
    imgs = torch.randint(0, 256, (32, 3, 224, 224), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 1000, (32,), generator=g)
    lc = cpu(imgs, labels)["loss"]
    lc.backward()
    lg = gpu(imgs.cuda(), labels.cuda())["loss"]
    lg.backward()
    torch.cuda.synchronize()
    _compare_leaves(cpu, gpu, lc, lg)


def test_paired_wgrads_match_separate():
    """Fused-block backward with consecutive weight gradients (FF2 + FF1, Wo + QKV) launched as
    grouped TN grids (ops/prims.py paired_wgrads) and the batched jumbo W1 + W2 gradients as one
    grouped segmented grid == every weight gradient on its own: same
    gradients up to fp32 summation order, same DP ``ready`` notifications per parameter."""
    from collections import Counter
    from jumbo_mae_tpu_amd.config import DecoderConfig, ViTConfig
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.ops import prims as P
    vc = ViTConfig(layers=2, dim=256, heads=4, labels=0, image_size=224, patch_size=16, posemb="sincos2d",
                   layerscale=True)
    dc = DecoderConfig(dec_layers=2, dec_dim=256, dec_heads=4, image_size=224, patch_size=16)
    m = PretrainModel(vc, dc).to("cuda", torch.bfloat16, seed=0)
    # 6656 encoder / 25472 decoder rows (TN path); 128-row jumbo blocks (grouped segmented W1 + W2)
    imgs = torch.randint(0, 256, (128, 3, 224, 224), dtype=torch.uint8, device="cuda")
    noise = torch.rand(196, device="cuda")
    grads, readies = [], []
    saved = P.PAIR_WGRAD, P.GROUP_JUMBO_WGRAD
    try:
        for pair in (False, True):
            P.PAIR_WGRAD = P.GROUP_JUMBO_WGRAD = pair
            seen = Counter()
            m.store.hooks.append(lambda h: seen.update([h.start]))
            m.store.zero_grad()
            m(imgs, noise=noise)["loss"].backward()
            torch.cuda.synchronize()
            m.store.hooks.pop()
            assert P._pair["held"] is None and P._pair["depth"] == 0
            grads.append(m.store.grad.clone())
            readies.append(seen)
    finally:
        P.PAIR_WGRAD, P.GROUP_JUMBO_WGRAD = saved
    assert readies[0] == readies[1] and sum(readies[0].values()) > 0
    a, b = grads
    assert ((a - b).norm() / a.norm()).item() < 1e-5
    for s in m.store.segments:
        x, y = a[s.offset:s.offset + s.numel], b[s.offset:s.offset + s.numel]
        assert (x - y).abs().max().item() <= 1e-4 * max(x.abs().max().item(), 1e-6), s.key


def test_store_mode_grads_match_zeroed():
    """Store-mode gradients (ParamStore.zero_grad leaves the TN-path Dense kernels to their first,
    storing write; the rest is zeroed by one multi-range launch) == zeroing the whole buffer, over
    two steps (the first registers the handles) with gradient accumulation (2 micro-steps)."""
    import jumbo_mae_tpu_amd.models.params as PM
    from jumbo_mae_tpu_amd.config import DecoderConfig, ViTConfig
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    vc = ViTConfig(layers=2, dim=256, heads=4, labels=0, image_size=224, patch_size=16, posemb="sincos2d",
                   layerscale=True)
    dc = DecoderConfig(dec_layers=2, dec_dim=256, dec_heads=4, image_size=224, patch_size=16)
    imgs = torch.randint(0, 256, (128, 3, 224, 224), dtype=torch.uint8, device="cuda")
    noise = torch.rand(196, device="cuda")
    out = []
    saved = PM.STORE_GRADS
    try:
        for store in (False, True):
            PM.STORE_GRADS = store
            m = PretrainModel(vc, dc).to("cuda", torch.bfloat16, seed=0)
            for _ in range(2):  # step 1 registers the store-mode handles, step 2 uses them
                m.store.grad.fill_(1e3)  # stale values: whatever zero_grad skips must be overwritten
                m.store.zero_grad()
                for _ in range(2):  # two micro-steps: the second accumulates
                    m(imgs, noise=noise)["loss"].backward()
                m.store.flush_fresh()
            torch.cuda.synchronize()
            out.append((m.store.grad.clone(), len(m.store._store_handles)))
    finally:
        PM.STORE_GRADS = saved
    (a, n0), (b, n1) = out
    assert n0 == 0 and n1 > 0
    assert torch.isfinite(b).all()
    assert ((a - b).norm() / a.norm()).item() < 1e-5
