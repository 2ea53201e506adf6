"""ZeRO-1 optimizer sharding (parallel/ddp.py ``shard=True``) on CPU gloo ranks: reduce-scatter of
the gradient buckets, update of this rank's pieces only, all-gather of the updated master.  The
result must be the replicated all-reduce step's, for every optimizer (per-leaf LAMB / LARS trust
ratios and the global clip norm are summed over the ranks), with the split (per-bucket) and the
monolithic update, and the gathered optimizer moments must equal the replicated ones."""

import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_dist import _cfgs, _free_port, _init


def _worker(rank, world, port, out, kind, clip, overlap, bf16, defer=False):
    _init(rank, world, port)
    from jumbo_mae_tpu_amd.ops import prims
    prims._deferred["force"] = defer  # batched jumbo wgrad in row chunks with partial readiness (GPU path)
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.optim.flat import FlatOptimizer
    from jumbo_mae_tpu_amd.optim.schedule import warmup_cosine_decay_schedule
    from jumbo_mae_tpu_amd.parallel.ddp import GradReducer
    from jumbo_mae_tpu_amd.train.engine import Trainer
    vc, dc = _cfgs()
    g = torch.Generator().manual_seed(0)
    imgs = torch.randint(0, 256, (4 * world, 3, 32, 32), dtype=torch.uint8, generator=g)
    res = {}
    for shard in (False, True):
        torch.manual_seed(100 + rank)  # same masking noise in both runs
        m = PretrainModel(vc, dc).to("cpu", seed=0)
        dist.broadcast(m.store.master, 0)
        opt = FlatOptimizer(m.store, kind, warmup_cosine_decay_schedule(1e-6, 1e-2, 1, 10, 1e-5), b2=0.95,
                            weight_decay=0.05, num_layers=vc.layers, clip_grad=clip)
        red = GradReducer(m.store, bucket_mb=0.01, shard=shard,
                          reduce_dtype=torch.bfloat16 if bf16 else torch.float32)
        tr = Trainer(m, opt, red, None)
        tr.overlap_optimizer = overlap
        early = []
        fin = red.finish

        def finish(*a, _fin=fin, _red=red, **k):  # buckets launched during the backward
            early.append([b for b, done in enumerate(_red.launched) if done])
            return _fin(*a, **k)

        red.finish = finish
        for _ in range(3):
            tr.train_step([(imgs[rank * 4:(rank + 1) * 4],)])
        opt.gather_state()
        res[shard] = {"master": m.store.master.clone(), "mu": None if opt.mu is None else opt.mu.clone(),
                      "trace": None if opt.trace is None else opt.trace.clone(), "stats": red.stats(),
                      "nb": len(red.buckets), "pieces": red.owned_pieces(), "early": early[-1],
                      "jumbo": [b for b, (lo, hi, idxs) in enumerate(red.buckets)
                                if any("jumbo_mlp" in red.segs[i].path and red.segs[i].numel > 1000 for i in idxs)]}
    # every rank ends with the same master
    ms = [torch.zeros_like(res[True]["master"]) for _ in range(world)]
    dist.all_gather(ms, res[True]["master"])
    if rank == 0:
        torch.save({"rep": res[False], "zero": res[True], "same": all(torch.equal(ms[0], x) for x in ms)}, out)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,kind,clip,overlap,bf16,defer", [
    (2, "adamw", 0.0, True, False, False),   # split update per bucket group + all-gather per group
    (2, "adamw", 0.0, False, False, False),  # monolithic update, then all-gather
    (2, "sgd", 0.0, True, False, False),
    (2, "lamb", 0.0, True, False, False),    # per-leaf trust ratios: norms summed over the ranks
    (2, "lars", 0.0, True, False, False),
    (2, "adamw", 0.5, True, False, False),   # global clip norm summed over the ranks
    (2, "adamw", 0.0, True, True, False),    # bf16 reduce-scatter
    (4, "adamw", 0.0, True, False, False),
    (4, "lamb", 0.3, True, False, False),
    (2, "adamw", 0.0, True, False, True),  # chunked jumbo weight gradients: sub-bucket reduce-scatters
    (4, "lamb", 0.0, True, True, True),
])
def test_zero1_matches_replicated(world, kind, clip, overlap, bf16, defer):
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.spawn(_worker, args=(world, port, out, kind, clip, overlap, bf16, defer), nprocs=world, join=True)
        r = torch.load(out, weights_only=True)
    rep, zero = r["rep"], r["zero"]
    assert r["same"], "ranks disagree after the all-gather"
    assert zero["stats"]["mode"] == "zero1-reduce-scatter" and rep["stats"]["mode"] == "all-reduce"
    assert zero["nb"] > 3
    # pieces: 64-aligned, one per bucket
    assert all(a % 64 == 0 and b % 64 == 0 and b > a for a, b in zero["pieces"])
    if defer:
        # each oversized jumbo kernel is cut into quarter sub-buckets, and all but the last of them
        # are reduce-scattered from their row chunks' partial readiness, before finish()
        jb = zero["jumbo"]
        assert len(jb) >= 8, jb
        assert len([b for b in jb if b in zero["early"]]) >= len(jb) - 2, (jb, zero["early"])
    if world == 2 and not bf16 and kind in ("adamw", "sgd") and clip == 0:
        # elementwise update, and two-rank sums are a single addition either way: bit for bit
        assert torch.equal(zero["master"], rep["master"])
        for k in ("mu", "trace"):
            if rep[k] is not None:
                assert torch.equal(zero[k], rep[k]), k
    else:
        # per-leaf / global norms summed as per-rank partials, gloo's 4-rank all-reduce and
        # reduce-scatter adding in different orders, bf16 rounding per rank: equal to rounding
        tol = 2e-3 if bf16 else 1e-5
        d = (zero["master"] - rep["master"]).abs().max().item()
        assert d <= tol * rep["master"].abs().max().item(), d
        if rep["mu"] is not None:
            d = (zero["mu"] - rep["mu"]).abs().max().item()
            assert d <= (4e-3 if bf16 else 1e-3) * rep["mu"].abs().max().item() + 1e-9, d


def _gather_worker(rank, world, port, out):
    _init(rank, world, port)
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.optim.flat import FlatOptimizer
    from jumbo_mae_tpu_amd.optim.schedule import warmup_cosine_decay_schedule
    from jumbo_mae_tpu_amd.parallel.ddp import GradReducer
    from jumbo_mae_tpu_amd.train.engine import Trainer
    vc, dc = _cfgs()
    g = torch.Generator().manual_seed(0)
    imgs = torch.randint(0, 256, (4 * world, 3, 32, 32), dtype=torch.uint8, generator=g)
    res = {}
    for gdt in ("fp32", "bf16"):
        torch.manual_seed(100 + rank)
        m = PretrainModel(vc, dc).to("cpu", torch.bfloat16, seed=0)  # bf16 compute: a separate shadow
        dist.broadcast(m.store.master, 0)
        m.store.sync_shadow()
        opt = FlatOptimizer(m.store, "adamw", warmup_cosine_decay_schedule(1e-6, 1e-2, 1, 10, 1e-5), b2=0.95,
                            weight_decay=0.05, num_layers=vc.layers)
        red = GradReducer(m.store, bucket_mb=0.01, shard=True, gather_dtype=gdt)
        assert red.gather_shadow == (gdt == "bf16")
        tr = Trainer(m, opt, red, None)
        for _ in range(3):
            tr.train_step([(imgs[rank * 4:(rank + 1) * 4],)])
        shadow = m.store.shadow.clone()  # before any master gather: what the next forward reads
        stale = not torch.equal(m.store.master.to(torch.bfloat16), shadow)
        opt.gather_state()  # checkpoint: the sharded master (bf16 mode) and moments made whole
        res[gdt] = {"shadow": shadow, "master": m.store.master.clone(), "mu": opt.mu.clone(), "stale": stale,
                    "stats": red.stats()}
    if rank == 0:
        torch.save(res, out)
    dist.destroy_process_group()


def test_zero1_bf16_shadow_gather_matches_fp32_gather():
    """ZeRO-1 all-gathering the bf16 shadow (default) vs the fp32 master + re-cast: the same weights
    bit for bit (shadow every step; master and moments after the checkpoint gather); with the bf16
    gather the master of non-owned pieces is stale until that gather."""
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.spawn(_gather_worker, args=(2, port, out), nprocs=2, join=True)
        r = torch.load(out, weights_only=True)
    f, b = r["fp32"], r["bf16"]
    assert f["stats"]["gather_dtype"] == "fp32" and b["stats"]["gather_dtype"] == "bf16"
    assert torch.equal(b["shadow"], f["shadow"])
    assert torch.equal(b["master"], f["master"]) and torch.equal(b["mu"], f["mu"])
    assert b["stale"] and not f["stale"]


def test_shard_ranges_tile_and_align():
    from jumbo_mae_tpu_amd.parallel.ddp import shard_ranges
    rs = shard_ranges([(1000, 5000), (5000, 5003), (5003, 9000), (9000, 20000)], 512)
    asc = sorted(rs)
    assert asc[0][0] == 512 and asc[-1][1] == 20480
    assert all(a % 512 == 0 and b % 512 == 0 and a < b for a, b in rs)
    assert all(x[1] == y[0] for x, y in zip(asc[:-1], asc[1:]))  # contiguous tiling
    assert rs == sorted(rs, reverse=True)  # launch order: from the end of the buffer
