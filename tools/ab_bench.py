"""Interleaved A/B of runtime switches on the flagship step (one process, one device).

    python tools/ab_bench.py --configs "blas:GEMM=blas" "auto:" --rounds 4 --steps 6

Each config is a list of ``KEY=VALUE`` switches applied to ``ops.prims`` module state between
rounds (same model, same data, same device -> no cross-process / cross-device variance).
Supported keys: GEMM (auto|blas|ours), DGRAD (0|1), WGRAD (0|1), WGRAD_STREAM (0|1),
and the Python-side constants below (kernel-level choices are fixed by shape in csrc/).
Prints per-config median / min ms per step."""

import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def apply(P, cfg: str):
    for kv in filter(None, cfg.split(",")):
        k, v = kv.split("=")
        if k == "GEMM":
            P._GEMM_MODE = v
        elif k == "DGRAD":
            P._DGRAD_OURS = v == "1"
        elif k == "WGRAD_STREAM":
            P.set_wgrad_stream(v == "1")
        elif k == "WGRAD":
            P._WGRAD_OURS = v == "1"
        elif k == "PAIR_WGRAD":  # 0: every weight gradient launched on its own
            P.PAIR_WGRAD = v == "1"
        elif k == "GROUP_JUMBO_WGRAD":  # 0: the jumbo W1 / W2 batched weight gradients launched apart
            P.GROUP_JUMBO_WGRAD = v == "1"
        elif k == "STORE_GRADS":  # 0: zero the whole gradient buffer every step
            import jumbo_mae_tpu_amd.models.params as PM
            PM.STORE_GRADS = v == "1"
        elif k == "WT_BATCH":
            import jumbo_mae_tpu_amd.models.params as PM
            PM.BATCH_TRANSPOSES = v == "1"
        elif k == "GELU_DERIV":
            P._GELU_DERIV = v == "1"
        elif k == "FWD_LINKS":
            from jumbo_mae_tpu_amd.ops import blocks
            blocks.FWD_LINKS = v == "1"
        elif k == "LINK_BLOCKS":
            from jumbo_mae_tpu_amd.ops import blocks
            blocks.LINKS = v == "1"
        elif k == "FUSE_LN_RES":
            P._FUSE_LN_RES = v == "1"
        elif k == "SEG_WGRAD":
            P._deferred["seg"] = v == "1"
        elif k == "DEFER_WGRAD":
            P._deferred["enabled"] = v == "1"
        elif k == "LN_FROM_H":  # 0: the LN backward reads the fp32 input instead of the bf16 output
            P._LN_BWD_FROM_H = v == "1"
        else:
            raise ValueError(k)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", required=True, help="name:KEY=V,KEY=V")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--model", default="vit_large_patch16")
    ap.add_argument("--batch", type=int, default=512, help="pretrain images per step (2048: the headline micro-batch)")
    ap.add_argument("--task", default="pretrain", choices=["pretrain", "finetune"],
                    help="finetune: the bench.py --task finetune step (ViT-B/16, config/ft.sh recipe, 128 images)")
    a = ap.parse_args()
    if a.task == "finetune":
        return run(a, finetune_step())
    from jumbo_mae_tpu_amd.config import decoder_config, vit_config
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.ops import prims as P
    from jumbo_mae_tpu_amd.optim.flat import FlatOptimizer
    from jumbo_mae_tpu_amd.train.engine import Trainer
    from jumbo_mae_tpu_amd.utils.rng import RngStreams
    dev = torch.device("cuda")
    vc = vit_config(a.model, labels=0, posemb="sincos2d", image_mask_ratio=0.75, droppath=0.0, dropout=0.0)
    dc = decoder_config(dec_droppath=0.0)
    model = PretrainModel(vc, dc).to(dev, torch.bfloat16, seed=0)
    opt = FlatOptimizer(model.store, "adamw", lambda c: 1e-4, b1=0.9, b2=0.95, weight_decay=0.05,
                        num_layers=vc.layers)
    tr = Trainer(model, opt, None, RngStreams({"noise": 0, "dropout": 0, "mixup": 0}, 0, dev))
    gen = torch.Generator(device=dev).manual_seed(0)
    pool = [torch.randint(0, 256, (a.batch, 3, 224, 224), dtype=torch.uint8, device=dev, generator=gen)
            for _ in range(2)]
    it = 0

    def step():
        nonlocal it
        tr.train_step([(pool[it % 2],)])
        it += 1

    run(a, (step, a.batch))


def finetune_step():
    """(step, images per step) of bench.py --task finetune at one rank."""
    from jumbo_mae_tpu_amd.train import common as C
    from jumbo_mae_tpu_amd.train.cli import finetune_parser
    from jumbo_mae_tpu_amd.train.engine import Trainer
    from jumbo_mae_tpu_amd.train.finetune import build_model
    from jumbo_mae_tpu_amd.utils.rng import RngStreams
    dev = torch.device("cuda")
    B, N = 128, 1281167
    flags = ["--mode", "finetune", "--layers", "12", "--dim", "768", "--heads", "12", "--labels", "1000",
             "--posemb", "sincos2d", "--droppath", "0.1", "--mixup", "0.8", "--cutmix", "1.0",
             "--label-smoothing", "0.1", "--optimizer", "adamw", "--learning-rate", "3e-3",
             "--weight-decay", "0.05", "--lr-decay", "0.75", "--warmup-steps", str(N * 10 // 1024),
             "--training-steps", str(N * 110 // 1024), "--train-batch-size", str(B)]
    for k in ("init", "mixup", "dropout", "shuffle", "noise"):
        flags += [f"--{k}-seed", "0"]
    fargs = finetune_parser().parse_args(flags)
    model = build_model(fargs, dev, torch.bfloat16, 0)
    model.store.sync_shadow()
    opt = C.make_optimizer(fargs, model.store, fargs.learning_rate, 1e-6)
    tr = Trainer(model, opt, None, RngStreams({"mixup": 1, "dropout": 1, "noise": 1}, 0, dev))
    gen = torch.Generator(device=dev).manual_seed(1234)
    pool = [(torch.randint(0, 256, (B, 3, 224, 224), dtype=torch.uint8, device=dev, generator=gen),
             torch.randint(0, 1000, (B,), device=dev, generator=gen)) for _ in range(2)]
    it = 0

    def step():
        nonlocal it
        tr.train_step([pool[it % 2]])
        it += 1

    return step, B


def run(a, step_b):
    from jumbo_mae_tpu_amd.ops import prims as P
    step, B = step_b
    cfgs = [c.split(":", 1) for c in a.configs]
    times = {n: [] for n, _ in cfgs}
    for r in range(a.rounds + 1):  # round 0 = warmup of every config
        for name, cfg in cfgs:
            apply(P, cfg)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize()
            if r > 0:
                times[name].append((time.perf_counter() - t0) * 1e3 / a.steps)
    for name, ts in times.items():
        print(f"{name:24s} median {statistics.median(ts):8.2f} ms  min {min(ts):8.2f} ms  "
              f"({B * 1e3 / statistics.median(ts):7.1f} img/s)  rounds {['%.1f' % t for t in ts]}", flush=True)


if __name__ == "__main__":
    main()
