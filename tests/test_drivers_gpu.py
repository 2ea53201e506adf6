"""The real product on the MI355X: the ``main_pretrain`` / ``main_finetune`` drivers end to end.

Reference workflow: ``main_pretrain`` writes ``{name}-last/-best.msgpack``
(/root/reference/src/main_pretrain.py:48-94, /root/reference/src/utils.py:55-63), then
``main_finetune --pretrained-ckpt`` loads its ``model`` subtree and trains a classifier end to end
(AdamW + layer-wise LR decay + Mixup / CutMix) or as a linear probe (LARS + BatchNorm head)
(/root/reference/src/main_finetune.py:48-94, /root/reference/src/finetuning.py:210-212,
/root/reference/src/utils.py:150-202).

Here every step of that chain runs on the GPU through the drivers themselves (``PT.main`` /
``FT.main`` with ``--device cuda``): real JPEG tar shards (data/jpeg_shards.py) read by the native
tar reader with 2 loader workers, decode + RandomResizedCrop + flip (+ RandAugment / random
erasing in finetuning), the ``DevicePrefetcher``'s pinned H2D copies, the sanity and periodic
``evaluate()`` on the GPU, the background msgpack writer, ``--resume auto`` and
``--pretrained-ckpt``.  Checks: losses decrease; the exported msgpack is the cuda master bit for
bit; an interrupted + resumed run ends bit-identical to an uninterrupted one; the finetune
model's encoder equals the checkpoint's ``model/*`` subtree after loading; the linear probe leaves
the encoder untouched (frozen) and trains the head."""

import json
import os

import numpy as np
import pytest
import torch

from jumbo_mae_tpu_amd.ckpt.checkpoint import load_params
from jumbo_mae_tpu_amd.ckpt.msgpack_flax import flatten_tree
from jumbo_mae_tpu_amd.data.jpeg_shards import write_shards
from jumbo_mae_tpu_amd.train import finetune as FT
from jumbo_mae_tpu_amd.train import pretrain as PT
from jumbo_mae_tpu_amd.train.cli import finetune_parser, pretrain_parser

pytestmark = pytest.mark.gpu

MODEL = ["--layers", "4", "--dim", "256", "--heads", "4", "--patch-size", "16", "--image-size", "224",
         "--posemb", "sincos2d"]
SEEDS = ["--init-seed", "0", "--mixup-seed", "0", "--dropout-seed", "0", "--noise-seed", "0", "--shuffle-seed", "0"]
COMMON = MODEL + SEEDS + ["--train-loader-workers", "2", "--valid-loader-workers", "2", "--log-file-only",
                          "--device", "cuda"]


@pytest.fixture(scope="module")
def shards(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("jpeg"))
    train = write_shards(d, shards=4, per_shard=96, classes=10, seed=0, prefix="train")
    valid = write_shards(d, shards=1, per_shard=64, classes=10, seed=1, prefix="valid")
    return train, valid


def _pretrain_args(shards, out, name, steps, extra=()):
    train, valid = shards
    return pretrain_parser().parse_args(COMMON + [
        "--train-dataset-shards", train, "--valid-dataset-shards", valid, "--train-batch-size", "32",
        "--valid-batch-size", "32", "--auto-augment", "none", "--random-erasing", "0", "--augment-repeats", "1",
        "--labels", "0", "--dec-layers", "2", "--dec-dim", "128", "--dec-heads", "4", "--learning-rate", "1.2e-2",
        "--adam-b2", "0.95", "--droppath", "0.1", "--dec-droppath", "0.1", "--training-steps", str(steps),
        "--warmup-steps", "2", "--log-interval", "2", "--eval-interval", str(steps // 2), "--output-dir", out,
        "--name", name, *extra])


def _capture(monkeypatch, module):
    """Patch ``module.build_model`` to hand the built model to the test."""
    got = []
    orig = module.build_model

    def build(*a, **k):
        m = orig(*a, **k)
        got.append(m)
        return m

    monkeypatch.setattr(module, "build_model", build)
    return got


def _rows(out, name):
    return [json.loads(line) for line in open(os.path.join(out, f"{name}-metrics.jsonl"))]


def _flat(path):
    return flatten_tree(load_params(path))


def _assert_trees_equal(a, b, what):
    assert set(a) == set(b), what
    for k in a:
        assert np.asarray(a[k]).dtype == np.asarray(b[k]).dtype, (what, k)
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), (what, "/".join(k))


@pytest.fixture(scope="module")
def pretrained(shards, tmp_path_factory):
    """One GPU pretraining run shared by the tests below: (output dir, model, result)."""
    out = str(tmp_path_factory.mktemp("pretrain"))
    mp = pytest.MonkeyPatch()
    got = _capture(mp, PT)
    try:
        res = PT.main(_pretrain_args(shards, out, "p", 12))
    finally:
        mp.undo()
    return out, got[0], res


def test_pretrain_driver_on_gpu(pretrained):
    out, model, res = pretrained
    assert model.store.master.is_cuda and model.store.shadow.dtype == torch.bfloat16
    rows = _rows(out, "p")
    vals = [r["val/loss"] for r in rows if "val/loss" in r]
    assert len(vals) == 3, rows  # sanity check at step 0, evals at 6 and 12
    print(f"[driver-test] val losses {vals}")
    # 12 steps of a toy model: 0.8006 -> 0.7469 -> 0.7378 (-7.8 %), the same to 6 digits with the exact gelu'
    # path (JMAE_GELU_CODES=0: 0.73780584 vs 0.73780632 with the 8-bit codes; profiles/r6e_driver_loss_codes.txt)
    assert vals[0] > vals[1] > vals[2] and vals[2] < 0.95 * vals[0], vals
    train = [r["train/loss"] for r in rows if "train/loss" in r]
    assert len(train) == 6 and all(np.isfinite(train)) and train[-1] < train[0], train
    assert any("perf/images_per_sec" in r for r in rows)
    for f in ("p-last.msgpack", "p-best.msgpack", "p-last.state.pt", "p-best.state.pt"):
        assert os.path.exists(os.path.join(out, f)), f
    assert res["final_step"] == 12
    # the exported msgpack is the cuda fp32 master bit for bit (last == final weights)
    live = flatten_tree(model.flax_params())
    _assert_trees_equal(_flat(os.path.join(out, "p-last.msgpack")), live, "last vs cuda master")
    for seg in model.store.segments[:5]:
        leaf = live[seg.path]
        assert np.array_equal(np.asarray(seg.from_flax(np.asarray(leaf))).reshape(-1),
                              model.store.master[seg.offset:seg.offset + seg.numel].cpu().numpy())


def test_resume_is_bitwise_on_gpu(shards, tmp_path):
    """An interrupted run (``--stop-after-steps 3``) resumed with ``--resume auto`` ends bit-identical
    to an uninterrupted one: weights, optimizer moments and the data stream (2 loader workers)."""
    out = str(tmp_path)
    PT.main(_pretrain_args(shards, out, "a", 6))
    PT.main(_pretrain_args(shards, out, "b", 6, ["--stop-after-steps", "3"]))
    mid = load_params(os.path.join(out, "b-last.msgpack"))
    PT.main(_pretrain_args(shards, out, "b", 6, ["--resume", "auto"]))
    a, b = _flat(os.path.join(out, "a-last.msgpack")), _flat(os.path.join(out, "b-last.msgpack"))
    assert any(not np.array_equal(np.asarray(v), np.asarray(b[k])) for k, v in flatten_tree(mid).items())
    _assert_trees_equal(a, b, "resumed vs uninterrupted")
    sa = torch.load(os.path.join(out, "a-last.state.pt"), weights_only=True)
    sb = torch.load(os.path.join(out, "b-last.state.pt"), weights_only=True)
    assert sa["step"] == sb["step"] == 6
    for k in ("mu", "nu"):
        assert torch.equal(sa["optimizer"][k], sb["optimizer"][k]), k
    la = [r["train/loss"] for r in _rows(out, "a") if "train/loss" in r]
    lb = [r["train/loss"] for r in _rows(out, "b") if "train/loss" in r]
    assert la[-1] == lb[-1], (la, lb)


def _finetune_args(shards, out, ckpt, mode, extra):
    train, valid = shards
    return finetune_parser().parse_args(COMMON + [
        "--mode", mode, "--pretrained-ckpt", ckpt, "--train-dataset-shards", train, "--valid-dataset-shards", valid,
        "--train-batch-size", "32", "--valid-batch-size", "32", "--augment-repeats", "1", "--labels", "10",
        "--training-steps", "12", "--warmup-steps", "2", "--log-interval", "2", "--eval-interval", "6",
        "--output-dir", out, "--name", "f", *extra])


def _check_loaded(model, ckpt_flat, snap):
    """Every encoder leaf of the checkpoint's ``model`` subtree is the model's, bit for bit, right
    after ``--pretrained-ckpt`` loading; the head keeps its fresh init."""
    enc = {k[1:]: v for k, v in ckpt_flat.items() if k[0] == "model"}
    mine = {k[1:]: v for k, v in snap.items() if k[0] == "model"}
    shared = [k for k in enc if k in mine and k[0] != "head"]
    assert len(shared) >= 0.9 * len(enc), (len(shared), len(enc))
    for k in shared:
        assert np.array_equal(np.asarray(enc[k], np.float32), np.asarray(mine[k])), "/".join(k)
    assert any(k[0] == "head" for k in mine)


def _capture_loaded(monkeypatch):
    got = _capture(monkeypatch, FT)
    snaps = []
    orig_build = FT.build_model

    def build(*a, **k):
        m = orig_build(*a, **k)
        load = m.store.load_flax_tree

        def load_and_snapshot(tree, *la, **lk):
            r = load(tree, *la, **lk)
            snaps.append(flatten_tree(m.flax_params()))
            return r

        m.store.load_flax_tree = load_and_snapshot
        return m

    monkeypatch.setattr(FT, "build_model", build)
    return got, snaps


def test_finetune_from_pretrained_on_gpu(pretrained, shards, tmp_path, monkeypatch):
    pdir, _, _ = pretrained
    ckpt = os.path.join(pdir, "p-last.msgpack")
    got, snaps = _capture_loaded(monkeypatch)
    res = FT.main(_finetune_args(shards, str(tmp_path), ckpt, "finetune", [
        "--optimizer", "adamw", "--learning-rate", "1e-3", "--lr-decay", "0.75", "--mixup", "0.8", "--cutmix", "1.0",
        "--label-smoothing", "0.1", "--droppath", "0.1", "--auto-augment", "rand-m9-mstd0.5-inc1",
        "--random-erasing", "0.25"]))
    assert len(snaps) == 1
    _check_loaded(got[0], _flat(ckpt), snaps[0])
    rows = _rows(str(tmp_path), "f")
    train = [r["train/loss"] for r in rows if "train/loss" in r]
    assert len(train) == 6 and all(np.isfinite(train)), train  # Mixup / CutMix targets: noisy
    vals = [r["val/loss"] for r in rows if "val/loss" in r]
    assert len(vals) == 3 and vals[-1] < vals[0], vals  # clean validation images: learns
    assert 0.0 <= res["val/acc1"] <= res["val/acc5"] <= 1.0
    assert os.path.exists(os.path.join(str(tmp_path), "f-last.msgpack"))
    live = flatten_tree(got[0].flax_params())
    _assert_trees_equal(_flat(os.path.join(str(tmp_path), "f-last.msgpack")), live, "finetune last vs master")


def test_linear_probe_from_pretrained_on_gpu(pretrained, shards, tmp_path, monkeypatch):
    pdir, _, _ = pretrained
    ckpt = os.path.join(pdir, "p-last.msgpack")
    got, snaps = _capture_loaded(monkeypatch)
    res = FT.main(_finetune_args(shards, str(tmp_path), ckpt, "linear", [
        # peak LR = lr x B / 256 = 6.25, the reference probe's 0.1 x 16384 / 256 (LARS trust 1e-3)
        "--optimizer", "lars", "--learning-rate", "50", "--weight-decay", "0", "--mixup", "0", "--cutmix", "0",
        "--label-smoothing", "0", "--droppath", "0", "--auto-augment", "none", "--random-erasing", "0"]))
    model = got[0]
    assert model.cfg.batch_norm and len(snaps) == 1
    _check_loaded(model, _flat(ckpt), snaps[0])
    last = _flat(os.path.join(str(tmp_path), "f-last.msgpack"))
    before = snaps[0]
    # frozen encoder (stop-gradient): every encoder leaf is still the pretrained one; the head moved
    enc = [k for k in before if k[0] == "model" and k[1] != "head"]
    assert enc
    for k in enc:
        assert np.array_equal(np.asarray(last[k]), np.asarray(before[k])), "/".join(k)
    head = [k for k in before if k[:2] == ("model", "head")]
    assert any(not np.array_equal(np.asarray(last[k]), np.asarray(before[k])) for k in head)
    rows = _rows(str(tmp_path), "f")
    train = [r["train/loss"] for r in rows if "train/loss" in r]
    assert len(train) == 6 and all(np.isfinite(train)), train
    vals = [r["val/loss"] for r in rows if "val/loss" in r]
    assert len(vals) == 3 and vals[-1] < vals[0], vals
    assert 0.0 <= res["val/acc1"] <= res["val/acc5"] <= 1.0
    # the BatchNorm running statistics travel in the resume sidecar
    st = torch.load(os.path.join(str(tmp_path), "f-last.state.pt"), weights_only=True)
    assert "batch_stats" in st and torch.isfinite(st["batch_stats"]["mean"]).all()
