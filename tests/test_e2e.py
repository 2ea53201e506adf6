"""End-to-end drivers on CPU: the BASELINE plumbing config (ViT-Tiny/16-style 32x32 MAE pretrain,
world_size 1), finetune from the pretrained checkpoint, linear probe, resume."""

import json
import os

import pytest

from jumbo_mae_tpu_amd.train import finetune as FT
from jumbo_mae_tpu_amd.train import pretrain as PT
from jumbo_mae_tpu_amd.train.cli import finetune_parser, pretrain_parser

COMMON = ["--train-loader-workers", "0", "--valid-loader-workers", "0", "--random-erasing", "0",
          "--image-size", "32", "--patch-size", "8", "--layers", "2", "--dim", "64", "--heads", "4",
          "--init-seed", "0", "--mixup-seed", "0", "--dropout-seed", "0", "--noise-seed", "0",
          "--shuffle-seed", "0", "--log-file-only", "--device", "cpu"]


def _pretrain(out, steps, extra=()):
    args = pretrain_parser().parse_args(COMMON + [
        "--train-dataset-shards", "synthetic:64", "--valid-dataset-shards", "synthetic:16",
        "--train-batch-size", "16", "--valid-batch-size", "8", "--auto-augment", "none", "--augment-repeats", "1",
        "--labels", "0", "--dec-layers", "1", "--dec-dim", "32", "--dec-heads", "2", "--learning-rate", "5e-3",
        "--training-steps", str(steps), "--warmup-steps", "2", "--log-interval", "2", "--eval-interval", str(steps),
        "--output-dir", out, "--name", "p", "--droppath", "0.1", "--dec-droppath", "0.1", *extra])
    return PT.main(args)


def test_pretrain_loss_decreases_and_checkpoints(tmp_path):
    out = str(tmp_path)
    res = _pretrain(out, 12)
    rows = [json.loads(line) for line in open(os.path.join(out, "p-metrics.jsonl"))]
    vals = [r["val/loss"] for r in rows if "val/loss" in r]
    assert len(vals) == 2 and vals[-1] < vals[0]  # sanitation-check eval vs final eval
    assert res["val/loss"] > 0
    for f in ("p-last.msgpack", "p-best.msgpack", "p-last.state.pt"):
        assert os.path.exists(os.path.join(out, f))


def test_resume(tmp_path):
    out = str(tmp_path)
    _pretrain(out, 4)
    res = _pretrain(out, 6, ["--resume", "auto"])
    rows = [json.loads(line) for line in open(os.path.join(out, "p-metrics.jsonl"))]
    steps = [r["step"] for r in rows if "train/loss" in r]
    assert steps[-1] == 6 and 2 in steps and 6 in steps
    assert res["final_step"] == 6


@pytest.mark.parametrize("mode,opt,lr", [("finetune", "adamw", "1e-3"), ("linear", "lars", "0.1"),
                                         ("linear", "sgd", "0.5")])
def test_finetune_and_linear(tmp_path, mode, opt, lr):
    out = str(tmp_path)
    _pretrain(out, 2)
    extra = ["--mixup", "0.8", "--cutmix", "1.0", "--auto-augment", "rand-m9-mstd0.5-inc1", "--lr-decay", "0.75"] \
        if mode == "finetune" else ["--mixup", "0", "--cutmix", "0", "--auto-augment", "none", "--droppath", "0"]
    args = finetune_parser().parse_args(COMMON + [
        "--mode", mode, "--optimizer", opt, "--learning-rate", lr, "--pretrained-ckpt", os.path.join(out, "p-last.msgpack"),
        "--train-dataset-shards", "synthetic:64:5", "--valid-dataset-shards", "synthetic:16:5",
        "--train-batch-size", "16", "--valid-batch-size", "8", "--augment-repeats", "1", "--labels", "5",
        "--posemb", "sincos2d", "--training-steps", "4", "--warmup-steps", "1", "--log-interval", "2",
        "--eval-interval", "4", "--output-dir", out, "--name", "f", *extra])
    res = FT.main(args)
    assert 0.0 <= res["val/acc1"] <= 1.0 and res["val/acc5"] >= res["val/acc1"]
    # reference semantics (main_finetune.py:86-88): "best" is written when val/acc1 beats the running
    # maximum, which starts at 0
    assert os.path.exists(os.path.join(out, "f-best.msgpack")) == (res.get("val/acc1/best", 0.0) > 0)
    assert os.path.exists(os.path.join(out, "f-last.msgpack"))


def test_skip_nonfinite_step_leaves_weights_untouched():
    """--skip-nonfinite: a step whose loss is NaN applies no update."""
    import torch

    from jumbo_mae_tpu_amd.config import DecoderConfig, ViTConfig
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.optim.flat import FlatOptimizer
    from jumbo_mae_tpu_amd.train.engine import Trainer
    vc = ViTConfig(layers=1, dim=32, heads=4, labels=0, image_size=32, patch_size=8, posemb="sincos2d")
    dc = DecoderConfig(dec_layers=1, dec_dim=16, dec_heads=2, image_size=32, patch_size=8)
    m = PretrainModel(vc, dc).to("cpu")
    opt = FlatOptimizer(m.store, "adamw", lambda c: 1e-3, weight_decay=0.05)
    tr = Trainer(m, opt, skip_nonfinite=True)
    imgs = torch.randint(0, 256, (2, 3, 32, 32), dtype=torch.uint8)
    tr.train_step([(imgs,)])
    assert tr.skipped_steps == 0
    with torch.no_grad():
        m.store.master[0] = float("nan")  # poisons the patch-embedding kernel -> NaN loss
    before = m.store.master.clone()
    tr.train_step([(imgs,)])
    assert tr.skipped_steps == 1
    assert torch.equal(torch.nan_to_num(m.store.master, nan=7.0), torch.nan_to_num(before, nan=7.0))
