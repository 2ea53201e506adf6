"""ZeRO-1 sharded optimizer kernels at world > 1, simulated on one GPU.

The multi-rank RCCL run is the driver's; here every rank of an N-rank job is replayed in turn on
the one device.  Rank r gets the chunk-table rows of exactly its owned pieces
(``FlatOptimizer._rows_for``), the HIP AdamW / SGD / LAMB / LARS kernels update copies of the
master and the moments, and the cross-rank SUM all-reduces of the per-leaf norms and the global
clip norm (``GradReducer.sum_``) are replaced by the sum of every rank's partials, computed by
running the ranks once per collective call.  The union of the owned pieces must equal the
unsharded update: bit for bit for the elementwise optimizers, to rounding for the norm-based ones
(LAMB, LARS, global-norm clipping: the chunk partials are summed in another grouping).  Nothing
outside a rank's pieces may change.  Pieces come from the reducer's own bucket planner
(``parallel/ddp.py`` plan_buckets + shard_ranges) at a small bucket size, so buckets cut
segments.  The bf16 shadow assembled from the owners' pieces -- what the default ZeRO-1 all-gather
(``gather_dtype="bf16"``) puts on every rank -- must equal the replicated step's shadow bit for bit.  Reference: /root/reference/src/pretraining.py:150 (pmean) + the optax update."""

import pytest
import torch

from jumbo_mae_tpu_amd.config import DecoderConfig, ViTConfig
from jumbo_mae_tpu_amd.models.mae import PretrainModel
from jumbo_mae_tpu_amd.models.params import ALIGN
from jumbo_mae_tpu_amd.optim.flat import FlatOptimizer
from jumbo_mae_tpu_amd.optim.schedule import warmup_cosine_decay_schedule
from jumbo_mae_tpu_amd.parallel.ddp import plan_buckets, shard_ranges, unit_key

pytestmark = pytest.mark.gpu


class _SimShard:
    """Stands in for a sharded GradReducer of one rank: owned pieces + scripted SUM all-reduces."""
    shard = True

    def __init__(self, pieces, totals):
        self.pieces, self.totals = pieces, totals
        self.calls, self.recorded = 0, None

    def owned_pieces(self, buckets=None):
        return self.pieces

    def sum_(self, t):
        i = self.calls
        self.calls += 1
        if i < len(self.totals):
            t.copy_(self.totals[i])
        elif i == len(self.totals):
            self.recorded = t.clone()


def _model():
    vc = ViTConfig(layers=2, dim=128, heads=2, labels=0, image_size=64, patch_size=16, posemb="sincos2d",
                   layerscale=True)
    dc = DecoderConfig(dec_layers=1, dec_dim=64, dec_heads=2, image_size=64, patch_size=16)
    return PretrainModel(vc, dc).to("cuda", torch.bfloat16, seed=0)


def _pieces(store, world, bucket_elems=6000):
    segs = [s for s in store.segments if s.trainable]
    buckets = plan_buckets([s.numel for s in segs], [unit_key(s.path) for s in segs], bucket_elems)
    ranges = [(min(segs[i].offset for i in b), max(segs[i].offset + segs[i].numel for i in b)) for b in buckets]
    q = world * ALIGN
    assert store.total % q == 0
    shards = shard_ranges(ranges, q)
    per_rank = [[] for _ in range(world)]
    for lo, hi in shards:
        n = (hi - lo) // world
        for r in range(world):
            per_rank[r].append((lo + r * n, lo + (r + 1) * n))
    return shards, per_rank


def _opt(store, kind, clip):
    sched = warmup_cosine_decay_schedule(2e-2, 2e-2, 1, 10, 1e-3)
    return FlatOptimizer(store, kind, sched, b1=0.9, b2=0.95, weight_decay=0.05, lr_decay=0.8, num_layers=2,
                         clip_grad=clip)


def _state(opt):
    return [t for t in (opt.mu, opt.nu, opt.trace) if t is not None]


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("kind,clip,split", [("adamw", 0.0, False), ("adamw", 0.0, True), ("sgd", 0.0, True),
                                             ("lamb", 0.0, False), ("lars", 0.0, False),
                                             ("adamw", 0.05, False)])
def test_sharded_update_union_equals_replicated(world, kind, clip, split):
    m = _model()
    s = m.store
    gen = torch.Generator(device="cuda").manual_seed(7)
    s.grad.copy_(torch.randn(s.total, device="cuda", generator=gen) * 0.01)
    s.grad[s.used_numel():] = 0
    master0, grad0 = s.master.clone(), s.grad.clone()
    ref = _opt(s, kind, clip)
    state0 = [torch.rand(s.total, device="cuda", generator=gen) * 1e-4 for _ in _state(ref)]
    for t, v in zip(_state(ref), state0):
        t.copy_(v)
    ref.step()
    torch.cuda.synchronize()
    want_master, want_shadow = s.master.clone(), s.shadow.clone()
    want_state = [t.clone() for t in _state(ref)]

    shards, per_rank = _pieces(s, world)
    assert len(shards) >= 4  # several buckets, boundaries cutting segments

    def run_rank(r, totals):
        s.master.copy_(master0)
        s.shadow.zero_()
        s.grad.copy_(grad0)
        opt = _opt(s, kind, clip)
        for t, v in zip(_state(opt), state0):
            t.copy_(v)
        sim = _SimShard(per_rank[r], totals)
        opt.attach_shard(sim)
        if split:  # the per-bucket-group path GradReducer.finish drives (on_bucket_done -> launch_range)
            groups = [shards[: len(shards) // 2], shards[len(shards) // 2:]]
            ranges = [(min(lo for lo, _ in g), max(hi for _, hi in g)) for g in groups]
            pieces = [[p for p in per_rank[r] if lo <= p[0] < hi] for lo, hi in ranges]
            opt.prepare()
            opt.plan_ranges(ranges, pieces)
            for lo, hi in ranges:
                opt.launch_range(lo, hi)
            opt.launch_rest()
            opt.finish()
        else:
            opt.step()
        torch.cuda.synchronize()
        return sim, s.master.clone(), s.shadow.clone(), [t.clone() for t in _state(opt)], s.grad.clone()

    # one pass per collective call: pass k runs every rank with the sums of calls < k known and
    # records its partial for call k
    totals = []
    while True:
        recs = [run_rank(r, totals)[0].recorded for r in range(world)]
        if recs[0] is None:
            assert all(x is None for x in recs)
            break
        totals.append(torch.stack(recs).sum(0))
    assert len(totals) == (int(clip > 0) + int(kind in ("lamb", "lars")))

    got_master, got_state = master0.clone(), [v.clone() for v in state0]
    # what the bf16-shadow all-gather assembles on every rank: each owner's shadow pieces
    got_shadow = torch.zeros_like(s.shadow)
    for r in range(world):
        _, mr, sh, st, gr = run_rank(r, totals)
        own = torch.zeros(s.total, dtype=torch.bool, device="cuda")
        for a, b in per_rank[r]:
            own[a:b] = True
        # nothing outside the owned pieces moves; the gradient is read-only
        assert torch.equal(mr[~own], master0[~own]), f"rank {r} wrote outside its pieces"
        for t, v in zip(st, state0):
            assert torch.equal(t[~own], v[~own])
        assert torch.equal(gr, grad0)
        # the kernel's bf16 shadow of the owned pieces is the cast of the new master
        assert torch.equal(sh[own], mr[own].to(torch.bfloat16))
        got_master[own] = mr[own]
        got_shadow[own] = sh[own]
        for g, t in zip(got_state, st):
            g[own] = t[own]
    used = torch.zeros(s.total, dtype=torch.bool, device="cuda")
    for seg in s.segments:
        if seg.trainable:
            used[seg.offset:seg.offset + seg.numel] = True
    covered = torch.zeros_like(used)
    for r in range(world):
        for a, b in per_rank[r]:
            covered[a:b] = True
    assert bool(covered[used].all()), "owned pieces do not cover every trainable element"
    if kind in ("adamw", "sgd") and clip == 0:
        assert torch.equal(got_master[used], want_master[used])
        for g, w in zip(got_state, want_state):
            assert torch.equal(g[used], w[used])
        assert torch.equal(got_master[used].to(torch.bfloat16), want_shadow[used])
        # ZeRO-1's bf16 gather == the fp32 gather + re-cast == the replicated step, bit for bit
        assert torch.equal(got_shadow[used], want_shadow[used])
    else:
        delta = (want_master - master0)[used].abs().max().item()
        assert delta > 0
        torch.testing.assert_close(got_master[used], want_master[used], rtol=0, atol=max(1e-4 * delta, 1e-9))
        for g, w in zip(got_state, want_state):
            torch.testing.assert_close(g[used], w[used], rtol=1e-5, atol=1e-12)
