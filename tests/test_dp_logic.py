"""Single-process checks of the data-parallel machinery: per-rank
RNG streams, bucket partition and readiness-driven launch order of the gradient reducer (with a
fake collective), gradient-accumulation equivalence, linear probe reducing the head only."""

import torch

from jumbo_mae_tpu_amd.config import DecoderConfig, ViTConfig
from jumbo_mae_tpu_amd.utils.rng import RngStreams


def test_rng_streams_distinct_per_rank_and_deterministic():
    draws = {}
    for rank in range(3):
        r = RngStreams({"noise": 5, "dropout": 5, "mixup": 5}, rank, "cpu")
        draws[rank] = {k: torch.rand(8, generator=r.get(k)) for k in ("noise", "dropout", "mixup")}
    again = RngStreams({"noise": 5, "dropout": 5, "mixup": 5}, 1, "cpu")
    assert torch.equal(torch.rand(8, generator=again.get("noise")), draws[1]["noise"])
    flat = [v for d in draws.values() for v in d.values()]
    for i in range(len(flat)):
        for j in range(i + 1, len(flat)):
            assert not torch.equal(flat[i], flat[j])
    # consecutive draws of one stream differ (steps advance the generator)
    r = RngStreams({"noise": 5}, 0, "cpu")
    assert not torch.equal(torch.rand(8, generator=r.get("noise")), torch.rand(8, generator=r.get("noise")))


def _pretrain_model():
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    vc = ViTConfig(layers=3, dim=32, heads=4, labels=0, image_size=32, patch_size=8, posemb="sincos2d",
                   layerscale=True)
    dc = DecoderConfig(dec_layers=2, dec_dim=16, dec_heads=2, image_size=32, patch_size=8)
    return PretrainModel(vc, dc).to("cpu", seed=0)


class _FakeWork:
    def wait(self):
        pass


def test_reducer_buckets_partition_and_launch_in_readiness_order():
    from jumbo_mae_tpu_amd.parallel.ddp import GradReducer

    m = _pretrain_model()
    red = GradReducer(m.store, bucket_mb=0.02)  # tiny buckets: many of them
    segs = red.segs
    covered = sorted(i for _, _, idxs in red.buckets for i in idxs)
    assert covered == list(range(len(segs)))  # every trainable segment in exactly one bucket
    for lo, hi, idxs in red.buckets:  # one contiguous slice of the flat buffer (alignment pads only)
        assert all(lo <= segs[i].offset and segs[i].offset + segs[i].numel <= hi for i in idxs)
        assert hi - lo - sum(segs[i].numel for i in idxs) < 64 * (len(idxs) + 1)
    ranges = [(lo, hi) for lo, hi, _ in red.buckets]
    assert ranges == sorted(ranges, reverse=True)  # cut from the end: reverse of forward order
    assert all(a[0] >= b[1] for a, b in zip(ranges, ranges[1:]))  # disjoint
    # emulate a multi-rank run: enable overlap and record launches instead of RCCL calls
    launched = []
    red.enabled = red.overlap = True
    m.store.hooks.append(red._on_ready)
    m.store.use_hooks.append(red._on_use)
    red._allreduce = lambda t: (launched.append(t.data_ptr()), (_FakeWork(), None))[1]
    red.world = 2
    m.store.zero_grad()
    red.begin_step()
    g = torch.Generator().manual_seed(0)
    imgs = torch.randint(0, 256, (4, 3, 32, 32), dtype=torch.uint8, generator=g)
    m(imgs, noise=torch.rand(16, generator=g))["loss"].backward()
    early = list(launched)
    red.finish()
    assert len(early) == len(red.buckets), "all buckets must be launched by readiness during backward"
    assert sorted(launched) == sorted(set(launched))
    # decoder-side buckets (end of the buffer) become ready before the encoder's first layers
    base = m.store.grad.data_ptr()
    offs = [(p - base) // 4 for p in early]
    assert offs[0] > offs[-1]


def test_grad_accumulation_equivalence():
    """Two micro-batches of B/2 with grad_accum=2 == one batch of B (deterministic finetune
    config: no mixup / droppath)."""
    from jumbo_mae_tpu_amd.models.classifier import FinetuneModel
    from jumbo_mae_tpu_amd.optim.flat import FlatOptimizer
    from jumbo_mae_tpu_amd.optim.schedule import warmup_cosine_decay_schedule
    from jumbo_mae_tpu_amd.train.engine import Trainer

    vc = ViTConfig(layers=2, dim=32, heads=4, labels=7, image_size=32, patch_size=8, posemb="learnable")
    g = torch.Generator().manual_seed(1)
    imgs = torch.randint(0, 256, (8, 3, 32, 32), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 7, (8,), generator=g)
    outs = []
    for accum in (1, 2):
        m = FinetuneModel(vc).to("cpu", seed=0)
        opt = FlatOptimizer(m.store, "adamw", warmup_cosine_decay_schedule(1e-6, 1e-3, 1, 10, 1e-6),
                            weight_decay=0.05, num_layers=vc.layers)
        tr = Trainer(m, opt, None, None, grad_accum=accum)
        micro = [(imgs, labels)] if accum == 1 else [(imgs[:4], labels[:4]), (imgs[4:], labels[4:])]
        met = tr.train_step(micro)
        outs.append((met["loss"].item(), m.store.master.clone()))
    assert abs(outs[0][0] - outs[1][0]) < 1e-5
    assert torch.allclose(outs[0][1], outs[1][1], atol=1e-6)


def test_linear_probe_reducer_covers_head_only():
    from jumbo_mae_tpu_amd.models.classifier import FinetuneModel
    from jumbo_mae_tpu_amd.parallel.ddp import GradReducer

    vc = ViTConfig(layers=2, dim=32, heads=4, labels=10, image_size=32, patch_size=8, posemb="sincos2d",
                   linear_probing=True, batch_norm=True)
    m = FinetuneModel(vc).to("cpu", seed=0)
    red = GradReducer(m.store)
    total = sum(hi - lo for lo, hi, _ in red.buckets)
    J = 3 * 32
    assert total == 2 * J + J * 10 + 10  # BatchNorm scale/bias + Dense kernel/bias
    assert all(s.path[:2] == ("model", "head") for s in red.segs)


def test_bucket_plan_layer_aligned():
    """Buckets never split a layer unless the layer alone exceeds the size; an oversized segment
    is a bucket of its own (keeps partial launches); launch order is from the end of the buffer."""
    from jumbo_mae_tpu_amd.parallel.ddp import GradReducer, plan_buckets, unit_key

    assert unit_key(("model", "layer_3", "attn", "wq", "kernel")) == ("model", "layer_3")
    assert unit_key(("decoder_model", "dec_layer_0", "ff", "w1", "bias")) == ("decoder_model", "dec_layer_0")
    assert unit_key(("model", "jumbo_mlp", "w1", "kernel")) == ("model", "jumbo_mlp")
    assert unit_key(("decoder_proj", "kernel")) == ("decoder_proj", "kernel")
    keys = [("a",), ("l0",), ("l0",), ("l1",), ("l1",), ("j",), ("j",), ("j",)]
    sizes = [5, 4, 4, 4, 4, 30, 1, 2]
    b = plan_buckets(sizes, keys, 10)
    assert b == [[7, 6], [5], [4, 3], [2, 1], [0]]
    # ViT-L-like: one encoder layer per 64 MiB bucket, the jumbo kernels alone
    m = _pretrain_model()
    red = GradReducer(m.store, bucket_mb=0.05)
    for lo, hi, idxs in red.buckets:
        units = {unit_key(red.segs[i].path) for i in idxs}
        if len(units) > 1:  # several whole units
            for u in units:
                members = [i for i, s in enumerate(red.segs) if unit_key(s.path) == u]
                assert set(members) <= set(idxs), u

