"""List host<->device synchronizations inside a train step (torch.cuda.set_sync_debug_mode).

    python tools/sync_check.py --task pretrain|finetune|linear
Runs 2 warmup steps, then one step with sync debug mode "warn" and prints each syncing call site."""

import argparse
import os
import sys
import traceback
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", default="finetune")
    a = ap.parse_args()
    from jumbo_mae_tpu_amd.train import common as C
    from jumbo_mae_tpu_amd.train.cli import finetune_parser
    from jumbo_mae_tpu_amd.train.engine import Trainer
    from jumbo_mae_tpu_amd.train.finetune import build_model
    from jumbo_mae_tpu_amd.utils.rng import RngStreams
    dev = torch.device("cuda:0")
    if a.task == "pretrain":
        from jumbo_mae_tpu_amd.config import decoder_config, vit_config
        from jumbo_mae_tpu_amd.models.mae import PretrainModel
        from jumbo_mae_tpu_amd.optim.flat import FlatOptimizer
        from jumbo_mae_tpu_amd.optim.schedule import warmup_cosine_decay_schedule
        vc = vit_config("vit_base_patch16", labels=0, posemb="sincos2d", image_mask_ratio=0.75)
        model = PretrainModel(vc, decoder_config()).to(dev, torch.bfloat16, seed=0)
        opt = FlatOptimizer(model.store, "adamw", warmup_cosine_decay_schedule(1e-6, 1e-3, 10, 100, 1e-5),
                            b2=0.95, weight_decay=0.05, num_layers=vc.layers)
        batch = (torch.randint(0, 256, (64, 3, 224, 224), dtype=torch.uint8, device=dev),)
    else:
        flags = ["--mode", a.task, "--layers", "12", "--dim", "768", "--heads", "12", "--labels", "1000",
                 "--mixup", "0.8" if a.task == "finetune" else "0", "--cutmix", "1.0" if a.task == "finetune" else "0",
                 "--label-smoothing", "0.1", "--droppath", "0.1" if a.task == "finetune" else "0",
                 "--optimizer", "adamw" if a.task == "finetune" else "lars", "--lr-decay", "0.75",
                 "--train-batch-size", "64"]
        fargs = finetune_parser().parse_args(flags)
        model = build_model(fargs, dev, torch.bfloat16)
        opt = C.make_optimizer(fargs, model.store, 1e-3, 1e-6)
        batch = (torch.randint(0, 256, (64, 3, 224, 224), dtype=torch.uint8, device=dev),
                 torch.randint(0, 1000, (64,), device=dev))
    tr = Trainer(model, opt, None, RngStreams({}, 0, dev))
    for _ in range(2):
        tr.train_step([batch])
    torch.cuda.synchronize()
    seen = []

    def hook(message, category, filename, lineno, file=None, line=None):
        stack = "".join(traceback.format_stack(limit=12)[:-1])
        seen.append(f"{message}\n{stack}")

    warnings.showwarning = hook
    torch.cuda.set_sync_debug_mode("warn")
    tr.train_step([batch])
    torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    print(f"[sync_check] task={a.task}: {len(seen)} synchronizing calls in one step")
    for s in seen:
        print("----\n" + s)


if __name__ == "__main__":
    main()
