"""Correctness at the production shapes: the headline ViT-L/16 step at its 2048-image micro-batch
against the same 2048 images run as 4 x 512 accumulated micro-steps.

The math is identical -- the loss is the mean over images with one shared mask permutation (same
noise for every micro-step), so mean-of-4-means == the 2048 mean and the accumulated gradient is
the same sum -- but the kernels are routed differently: the 2048-image micro-batch puts the
N = 12288 jumbo GEMMs on 224-row 4-phase tiles instead of narrow tiles, the jumbo W1 data gradient
adds its fp32 addend through one split, the encoder GEMMs take other tile heights and the
LayerNorm / reduction grids are 4x larger; the 512-image micro-steps exercise store-mode first
writes followed by accumulation.  Every gradient leaf of the Flax tree must agree (cosine > 0.999)
and so must the loss (relative 1e-3).  Reference: gradient accumulation in
/root/reference/src/pretraining.py:132-158."""

import pytest
import torch

from jumbo_mae_tpu_amd.config import decoder_config, vit_config
from jumbo_mae_tpu_amd.models.mae import PretrainModel
from jumbo_mae_tpu_amd.ops.prims import join_wgrad_stream

pytestmark = pytest.mark.gpu


def _grads(model, batches, noise):
    s = model.store
    s.zero_grad()
    losses = []
    for i, imgs in enumerate(batches):
        model.micro_index = i
        out = model(imgs, rngs={}, det=False, noise=noise)
        (out["loss"] / len(batches)).backward()
        losses.append(out["loss"].detach().float())
    join_wgrad_stream()
    s.flush_fresh()
    torch.cuda.synchronize()
    return float(torch.stack(losses).mean()), s.grad.clone()


def test_vitl_2048_microbatch_equals_4x512_accumulation():
    torch.manual_seed(0)
    vc = vit_config("vit_large_patch16", labels=0, posemb="sincos2d", image_mask_ratio=0.75, droppath=0.0,
                    dropout=0.0)
    dc = decoder_config(dec_droppath=0.0)
    model = PretrainModel(vc, dc).to("cuda", torch.bfloat16, seed=0)
    gen = torch.Generator(device="cuda").manual_seed(11)
    imgs = torch.randint(0, 256, (2048, 3, 224, 224), dtype=torch.uint8, device="cuda", generator=gen)
    noise = torch.rand(vc.seq_patches, device="cuda", generator=gen)
    loss_big, g_big = _grads(model, [imgs], noise)
    loss_acc, g_acc = _grads(model, list(imgs.split(512)), noise)
    assert abs(loss_big - loss_acc) <= 1e-3 * abs(loss_big), (loss_big, loss_acc)
    worst = (2.0, None)
    checked = 0
    for seg in model.store.segments:
        if not seg.trainable:
            continue
        a = g_big[seg.offset:seg.offset + seg.numel].double()
        b = g_acc[seg.offset:seg.offset + seg.numel].double()
        assert torch.isfinite(a).all() and torch.isfinite(b).all(), seg.key
        if seg.key.endswith("attn/wk/bias"):
            # analytically zero (adding b_k shifts every score of a query row by q . b_k; softmax is
            # shift invariant): only rounding noise of ~1e-9 remains on both paths
            assert a.abs().max() < 1e-6 and b.abs().max() < 1e-6, seg.key
            continue
        na, nb = a.norm().item(), b.norm().item()
        if na == 0 and nb == 0:
            continue
        assert na > 0 and nb > 0, seg.key
        cos = float(a @ b) / (na * nb)
        worst = min(worst, (cos, seg.key))
        assert cos > 0.999 and abs(na / nb - 1) < 1e-2, (seg.key, cos, na, nb)
        checked += 1
    assert checked > 300, checked  # every ViT-L + decoder leaf
    print(f"[prod-shape] loss {loss_big:.6f} vs {loss_acc:.6f}; worst leaf cosine {worst[0]:.6f} ({worst[1]})")
