"""Activation checkpointing with random layers, data-parallel edge cases and exact resume (CPU).

* ``--grad-ckpt`` gives the same gradients as the plain run at droppath 0.1 / dropout 0.1 (the
  recompute replays the forward's droppath / dropout draws), and records each parameter use once
  (the DP reducer still launches buckets during backward).
* ``grad_accum > 1``: buckets launch during the last micro-step's backward (uses are counted on
  the synchronising micro-step only).
* ``--skip-nonfinite`` with 2 ranks where only one rank's loss is NaN: both ranks skip together.
* resume: per-rank RNG streams are saved / restored per rank; an interrupted + resumed run ends
  with exactly the parameters of an uninterrupted run (data position, RNG, optimizer, best metric).
"""

import json
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from jumbo_mae_tpu_amd.config import DecoderConfig, ViTConfig


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from jumbo_mae_tpu_amd.parallel import dist as pdist
    return pdist.init_distributed("cpu")


def _cfgs(ckpt, droppath=0.1, dropout=0.1):
    vc = ViTConfig(layers=2, dim=32, heads=4, labels=0, image_size=32, patch_size=8, posemb="sincos2d",
                   layerscale=True, droppath=droppath, dropout=dropout, grad_ckpt=ckpt)
    dc = DecoderConfig(dec_layers=2, dec_dim=16, dec_heads=2, image_size=32, patch_size=8, dec_droppath=droppath,
                       dec_dropout=dropout, grad_ckpt=ckpt)
    return vc, dc


def _pretrain_grads(ckpt, droppath, dropout):
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    vc, dc = _cfgs(ckpt, droppath, dropout)
    m = PretrainModel(vc, dc).to("cpu", seed=0)
    g = torch.Generator().manual_seed(1)
    imgs = torch.randint(0, 256, (4, 3, 32, 32), dtype=torch.uint8, generator=g)
    rngs = {"dropout": torch.Generator().manual_seed(5), "noise": torch.Generator().manual_seed(6)}
    m.store.zero_grad()
    loss = m(imgs, rngs=rngs)["loss"]
    loss.backward()
    return float(loss.detach()), m.store.grad.clone()


@pytest.mark.parametrize("droppath,dropout", [(0.1, 0.0), (0.1, 0.1), (0.5, 0.0)])
def test_grad_ckpt_matches_plain(droppath, dropout):
    l0, g0 = _pretrain_grads(False, droppath, dropout)
    l1, g1 = _pretrain_grads(True, droppath, dropout)
    assert l0 == l1
    rel = float((g1 - g0).norm() / g0.norm())
    assert rel < 1e-6, rel


def test_grad_ckpt_finetune_matches_plain():
    from jumbo_mae_tpu_amd.models.classifier import FinetuneModel

    def run(ckpt):
        vc = ViTConfig(layers=2, dim=32, heads=4, labels=5, image_size=32, patch_size=8, posemb="sincos2d",
                       droppath=0.1, dropout=0.1, grad_ckpt=ckpt)
        m = FinetuneModel(vc, label_smoothing=0.1).to("cpu", seed=0)
        imgs = torch.randint(0, 256, (4, 3, 32, 32), dtype=torch.uint8, generator=torch.Generator().manual_seed(2))
        labels = torch.tensor([0, 1, 2, 3])
        m.store.zero_grad()
        out = m.forward(imgs, labels, rngs={"dropout": torch.Generator().manual_seed(3)}, det=False)
        out["loss"].backward()
        return m.store.grad.clone()

    g0, g1 = run(False), run(True)
    assert float((g1 - g0).norm() / g0.norm()) < 1e-6


def test_grad_ckpt_counts_each_use_once():
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    vc, dc = _cfgs(True)
    m = PretrainModel(vc, dc).to("cpu", seed=0)
    uses, readies = {}, {}
    m.store.use_hooks.append(lambda h: uses.__setitem__(id(h), uses.get(id(h), 0) + 1))
    m.store.hooks.append(lambda h: readies.__setitem__(id(h), readies.get(id(h), 0) + 1))
    imgs = torch.randint(0, 256, (2, 3, 32, 32), dtype=torch.uint8)
    loss = m(imgs, rngs={"dropout": torch.Generator().manual_seed(0)})["loss"]
    loss.backward()
    assert uses and uses == {k: v for k, v in readies.items() if k in uses}


# ------------------------------------------------------------------- 2-rank gloo workers
def _overlap_worker(rank, world, port, out, ckpt, accum):
    _init(rank, world, port)
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.parallel.ddp import GradReducer
    vc, dc = _cfgs(ckpt)
    m = PretrainModel(vc, dc).to("cpu", seed=0)
    red = GradReducer(m.store, bucket_mb=0.01)
    early = []
    orig = red.finish

    def finish(*a, **k):
        early.append(sum(red.launched))
        return orig(*a, **k)

    red.finish = finish
    g = torch.Generator().manual_seed(rank)
    m.store.zero_grad()
    red.begin_step()
    for i in range(accum):
        red.set_sync(i == accum - 1)
        imgs = torch.randint(0, 256, (2, 3, 32, 32), dtype=torch.uint8, generator=g)
        m(imgs, rngs={"dropout": torch.Generator().manual_seed(rank)})["loss"].backward()
    red.set_sync(True)
    red.finish()
    if rank == 0:
        torch.save({"early": early[0], "nb": len(red.buckets)}, out)
    dist.destroy_process_group()


@pytest.mark.parametrize("ckpt,accum", [(True, 1), (False, 2), (True, 2)])
def test_buckets_launch_during_backward(tmp_path, ckpt, accum):
    out = str(tmp_path / "o.pt")
    mp.spawn(_overlap_worker, args=(2, _free_port(), out, ckpt, accum), nprocs=2, join=True)
    r = torch.load(out, weights_only=True)
    assert r["nb"] > 2
    assert r["early"] >= r["nb"] - 2, r  # all but the embedding-side buckets launched before finish()


def _skip_worker(rank, world, port, out):
    _init(rank, world, port)
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.optim.flat import FlatOptimizer
    from jumbo_mae_tpu_amd.parallel.ddp import GradReducer
    from jumbo_mae_tpu_amd.train.engine import Trainer
    vc, dc = _cfgs(False, 0.0, 0.0)
    m = PretrainModel(vc, dc).to("cpu", seed=0)
    opt = FlatOptimizer(m.store, "adamw", lambda c: 1e-3, weight_decay=0.05)
    tr = Trainer(m, opt, GradReducer(m.store, bucket_mb=1.0), skip_nonfinite=True)
    fwd = m.forward
    poison = {"on": False}

    def forward(*a, **k):
        o = fwd(*a, **k)
        if poison["on"] and rank == 1:  # only rank 1 sees a non-finite loss
            o["loss"] = o["loss"] * float("nan")
        return o

    m.forward = forward
    m.__class__.__call__ = lambda self, *a, **k: self.forward(*a, **k)
    imgs = torch.randint(0, 256, (2, 3, 32, 32), dtype=torch.uint8, generator=torch.Generator().manual_seed(rank))
    tr.train_step([(imgs,)])
    before = m.store.master.clone()
    poison["on"] = True
    tr.train_step([(imgs,)])
    after = m.store.master.clone()
    torch.save({"skipped": tr.skipped_steps, "unchanged": bool(torch.equal(before, after)),
                "finite": bool(torch.isfinite(after).all())}, f"{out}.{rank}")
    dist.destroy_process_group()


def test_skip_nonfinite_is_global(tmp_path):
    out = str(tmp_path / "s")
    mp.spawn(_skip_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        d = torch.load(f"{out}.{r}", weights_only=True)
        assert d == {"skipped": 1, "unchanged": True, "finite": True}, (r, d)


# ------------------------------------------------------------------------------ resume
def _rank_state_worker(rank, world, port, out):
    _init(rank, world, port)
    from jumbo_mae_tpu_amd.train import common as C
    from jumbo_mae_tpu_amd.utils.mixup import Mixup
    from jumbo_mae_tpu_amd.utils.rng import RngStreams

    class M:
        mixup = Mixup(0.8, 1.0, seed=rank)

    rngs = RngStreams({"mixup": 0, "dropout": 0, "noise": 0}, rank, "cpu")
    torch.rand(5, generator=rngs.get("noise"))
    states = C.rank_states(rngs, M())
    want = torch.rand(3, generator=rngs.get("noise"))
    # a fresh process state restored from the gathered list continues THIS rank's stream
    fresh = RngStreams({"mixup": 0, "dropout": 0, "noise": 0}, rank, "cpu")
    fresh.load_state_dict(states[rank]["rngs"])
    got = torch.rand(3, generator=fresh.get("noise"))
    torch.save({"n": len(states), "match": bool(torch.equal(want, got)), "draw": got}, f"{out}.{rank}")
    dist.destroy_process_group()


def test_rank_states_are_per_rank(tmp_path):
    out = str(tmp_path / "r")
    mp.spawn(_rank_state_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    d0, d1 = (torch.load(f"{out}.{r}", weights_only=True) for r in range(2))
    assert d0["n"] == d1["n"] == 2 and d0["match"] and d1["match"]
    assert not torch.equal(d0["draw"], d1["draw"])  # ranks keep independent streams


@pytest.mark.parametrize("workers", [0, 2])
def test_loader_resume_continues_stream(workers):
    """create_dataloaders(start_batches=k) yields exactly batches k, k+1, ... of a fresh loader."""
    import argparse

    from jumbo_mae_tpu_amd.data.loader import create_dataloaders
    args = argparse.Namespace(random_crop="rrc", image_size=16, auto_augment="rand-m9-mstd0.5-inc1",
                              color_jitter=0.0, random_erasing=0.25, test_crop_ratio=0.875,
                              train_dataset_shards="synthetic:40:5", mode="finetune", augment_repeats=2,
                              shuffle_seed=0, train_batch_size=4, grad_accum=1, train_loader_workers=workers,
                              valid_dataset_shards=None)
    full, _ = create_dataloaders(args)
    it = iter(full)
    ref = [next(it) for _ in range(7)]
    for start in (4, 3, 5):  # odd starts: the resumed loader's worker 0 continues the stream of worker 1
        resumed, _ = create_dataloaders(args, start_batches=start)
        it2 = iter(resumed)
        for k in range(start, 7):
            b = next(it2)
            assert torch.equal(b[0], ref[k][0]) and torch.equal(b[1], ref[k][1]), (start, k)


@pytest.mark.parametrize("stop", [4, 3])
def test_interrupted_run_resumes_exactly(tmp_path, stop):
    """6 steps uninterrupted == ``stop`` steps (--stop-after-steps) + --resume auto to 6: same weights.
    stop=3 saves at a step without an evaluation (eval interval 2): validation must not advance the
    training RNG streams, or the resumed run's streams diverge."""
    from jumbo_mae_tpu_amd.ckpt.checkpoint import load_params
    from tests.test_e2e import _pretrain
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    extra = ["--eval-interval", "2", "--augment-repeats", "2"]
    _pretrain(a, 6, extra)
    _pretrain(b, 6, extra + ["--stop-after-steps", str(stop)])
    rows = [json.loads(line) for line in open(os.path.join(b, "p-metrics.jsonl"))]
    assert max(r["step"] for r in rows) <= stop
    res = _pretrain(b, 6, extra + ["--resume", "auto"])
    assert res["final_step"] == 6
    pa, pb = load_params(os.path.join(a, "p-last.msgpack")), load_params(os.path.join(b, "p-last.msgpack"))

    def leaves(t, pre=()):
        for k, v in t.items():
            if isinstance(v, dict):
                yield from leaves(v, pre + (k,))
            else:
                yield pre + (k,), v

    la, lb = dict(leaves(pa)), dict(leaves(pb))
    assert la.keys() == lb.keys()
    for k in la:
        assert (la[k] == lb[k]).all(), k
    # the best validation loss survives the resume (not reset to +inf)
    rb = [json.loads(line) for line in open(os.path.join(b, "p-metrics.jsonl"))]
    ra = [json.loads(line) for line in open(os.path.join(a, "p-metrics.jsonl"))]
    best_a = [r["val/loss/best"] for r in ra if "val/loss/best" in r]
    best_b = [r["val/loss/best"] for r in rb if "val/loss/best" in r]
    assert best_a[-1] == best_b[-1]
