"""Loss-curve A/B of the saved FF1 derivative: gelu'(h) as 8-bit codes (ops/prims.py _GELU_DERIV,
the default fused path) against the exact path that saves h and recomputes gelu'(h) in the FF2
data-gradient epilogue (EPI_DGELU).  Same seeds, same data, same initial weights; the only
difference between the two runs is the gelu' numerics in the backward.

A third run takes the exact path with another mask / dropout seed: its distance to the first
exact run is the run-to-run noise scale the code-vs-exact distance is judged against.

Tasks (both on learnable synthetic data: smooth images = bilinearly upsampled 14 x 14 noise, so
masked patches are predictable from their neighbours; labels = argmax of a fixed random linear
map of the low-resolution field):
  pretrain   ViT-B/16 Jumbo-MAE + 8 x 512 decoder, AdamW, batch 256
  finetune   ViT-B/16 classifier (10 classes), AdamW + LLRD, droppath 0.1, dropout 0.1, batch 256

  python tools/gelu_code_ab.py --task pretrain --steps 600
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_data(n_batches, B, dev, seed=7, labels=10):
    g = torch.Generator(device=dev).manual_seed(seed)
    proj = torch.randn(labels, 3 * 14 * 14, device=dev, generator=g)
    out = []
    for _ in range(n_batches):
        z = torch.rand(B, 3, 14, 14, device=dev, generator=g)
        img = torch.nn.functional.interpolate(z, size=(224, 224), mode="bilinear", align_corners=False)
        y = (z.flatten(1) - 0.5) @ proj.t()
        out.append(((img * 255).round().clamp(0, 255).to(torch.uint8), y.argmax(1)))
    return out


def run_pretrain(codes, noise_seed, steps, data, dev):
    from jumbo_mae_tpu_amd.config import decoder_config, vit_config
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.ops import prims
    from jumbo_mae_tpu_amd.optim.flat import FlatOptimizer
    from jumbo_mae_tpu_amd.optim.schedule import warmup_cosine_decay_schedule
    from jumbo_mae_tpu_amd.train.engine import Trainer
    from jumbo_mae_tpu_amd.utils.rng import RngStreams

    prims._GELU_DERIV = codes
    vc = vit_config("vit_base_patch16", labels=0, posemb="sincos2d", image_mask_ratio=0.75, droppath=0.0,
                    dropout=0.0)
    dc = decoder_config(dec_droppath=0.0)
    model = PretrainModel(vc, dc).to(dev, torch.bfloat16 if dev.type == "cuda" else torch.float32, seed=0)
    model.store.sync_shadow()
    sched = warmup_cosine_decay_schedule(1e-6, 1e-3, steps // 10, steps, 1e-5)
    opt = FlatOptimizer(model.store, "adamw", sched, b1=0.9, b2=0.95, eps=1e-8, weight_decay=0.05,
                        num_layers=vc.layers)
    trainer = Trainer(model, opt, None, RngStreams({"noise": noise_seed, "dropout": noise_seed, "mixup": 0}, 0, dev))
    losses = []
    for i in range(steps):
        m = trainer.train_step([(data[i % len(data)][0],)])
        losses.append(m["loss"])
    return [float(x) for x in torch.stack(losses).cpu()]


def run_finetune(codes, noise_seed, steps, data, dev):
    from jumbo_mae_tpu_amd.ops import prims
    from jumbo_mae_tpu_amd.train import common as C
    from jumbo_mae_tpu_amd.train.cli import finetune_parser
    from jumbo_mae_tpu_amd.train.engine import Trainer
    from jumbo_mae_tpu_amd.train.finetune import build_model
    from jumbo_mae_tpu_amd.utils.rng import RngStreams

    prims._GELU_DERIV = codes
    flags = ["--mode", "finetune", "--layers", "12", "--dim", "768", "--heads", "12", "--labels", "10",
             "--posemb", "sincos2d", "--droppath", "0.1", "--dropout", "0.1", "--mixup", "0.0", "--cutmix", "0.0",
             "--label-smoothing", "0.1", "--optimizer", "adamw", "--learning-rate", "5e-4", "--weight-decay", "0.05",
             "--lr-decay", "0.75", "--warmup-steps", str(steps // 10), "--training-steps", str(steps),
             "--train-batch-size", str(data[0][0].shape[0])]
    for k in ("init", "mixup", "shuffle"):
        flags += [f"--{k}-seed", "0"]
    flags += ["--dropout-seed", str(noise_seed), "--noise-seed", str(noise_seed)]
    fargs = finetune_parser().parse_args(flags)
    model = build_model(fargs, dev, torch.bfloat16 if dev.type == "cuda" else torch.float32, 0)
    model.store.sync_shadow()
    import contextlib
    with contextlib.redirect_stdout(sys.stderr):
        opt = C.make_optimizer(fargs, model.store, fargs.learning_rate, 1e-6)
    trainer = Trainer(model, opt, None, RngStreams({"mixup": 0, "dropout": noise_seed, "noise": noise_seed}, 0, dev))
    losses = []
    for i in range(steps):
        m = trainer.train_step([data[i % len(data)]])
        losses.append(m["loss"])
    return [float(x) for x in torch.stack(losses).cpu()]


def dist(a, b, tail):
    """mean |a - b| / mean(b) over the last ``tail`` steps, and the max over all steps of the
    20-step moving-average difference"""
    import numpy as np
    a, b = np.asarray(a), np.asarray(b)
    mean_rel = float(np.abs(a[-tail:] - b[-tail:]).mean() / b[-tail:].mean())
    k = 20
    ma = np.convolve(a, np.ones(k) / k, "valid")
    mb = np.convolve(b, np.ones(k) / k, "valid")
    return mean_rel, float(np.abs(ma - mb).max() / mb.mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", default="pretrain", choices=["pretrain", "finetune"])
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--out", default="")
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    dev = torch.device(a.device)
    data = make_data(16, a.batch, dev)
    fn = run_pretrain if a.task == "pretrain" else run_finetune
    runs = {}
    for name, codes, seed in (("codes_s0", True, 0), ("exact_s0", False, 0), ("exact_s1", False, 1)):
        runs[name] = fn(codes, seed, a.steps, data, dev)
        print(f"[gelu_ab] {a.task} {name}: first {runs[name][0]:.4f} last {runs[name][-1]:.4f}", file=sys.stderr,
              flush=True)
    tail = max(20, a.steps // 5)
    res = {"task": a.task, "steps": a.steps, "batch": a.batch,
           "first_loss": runs["exact_s0"][0], "final_loss_tail_mean": {k: sum(v[-tail:]) / tail for k, v in runs.items()},
           "codes_vs_exact_same_seed": dist(runs["codes_s0"], runs["exact_s0"], tail),
           "exact_seed0_vs_seed1": dist(runs["exact_s1"], runs["exact_s0"], tail)}
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"summary": res, "curves": runs}, f)


if __name__ == "__main__":
    main()
