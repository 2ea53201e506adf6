"""Finetune / linear-probe driver (``main_finetune``).

Parity: /root/reference/src/main_finetune.py:37-94 and create_train_state
(/root/reference/src/finetuning.py:168-278):
  * ``--mode finetune``: end-to-end training with Mixup/CutMix, label smoothing, LLRD, droppath;
  * ``--mode linear``: frozen encoder (stop-gradient) + SyncBatchNorm + Dense head;
  * optimizers adamw | lamb | lars | sgd (momentum 0.9); peak LR = lr * B / 256 for LARS, raw lr
    otherwise; warmup-cosine from 1e-6 to 1e-6;
  * ``--pretrained-ckpt``: Flax msgpack; encoder subtree loaded into the fresh tree (Q6 fix);
  * best checkpoint by maximum ``val/acc1``.
"""

from __future__ import annotations

import time

import torch

from ..ckpt.checkpoint import load_pretrained_params
from ..config import ViTConfig
from ..data.loader import create_dataloaders
from ..models.classifier import FinetuneModel
from ..parallel import dist as pdist
from ..utils.flops import finetune_fwd_flops_per_image
from ..utils.mixup import Mixup
from ..utils.trace import set_enabled as set_trace_ranges
from ..utils.rng import RngStreams
from . import common as C
from .cli import finetune_parser
from ..runtime.graph import StepRunner
from .engine import Trainer
from .meter import AverageMeter, Logger


def build_model(args, device, dtype, rank: int = 0) -> FinetuneModel:
    linear = args.mode == "linear"
    vc = ViTConfig(layers=args.layers, dim=args.dim, heads=args.heads, labels=args.labels, layerscale=args.layerscale,
                   patch_size=args.patch_size, image_size=args.image_size, posemb=args.posemb, pooling=args.pooling,
                   dropout=args.dropout, droppath=args.droppath, grad_ckpt=args.grad_ckpt, image_mask_ratio=None,
                   linear_probing=linear, batch_norm=linear)
    mix = Mixup(args.mixup, args.cutmix, seed=args.mixup_seed * 1009 + rank)
    return FinetuneModel(vc, mix, args.label_smoothing, args.criterion).to(device, dtype, seed=args.init_seed)


def evaluate(model, loader, rngs, device) -> dict:
    rngs = rngs.fork()  # validation never advances the training streams
    sums = None
    for images, labels in C.DevicePrefetcher(loader, device):
        m = model.evaluate(images, labels, rngs.as_dict())
        sums = m if sums is None else {k: sums[k] + m[k] for k in m}
    keys = ["loss", "acc1", "acc5", "num_samples"]
    packed = torch.stack([sums[k].float() for k in keys])
    pdist.all_reduce_sum_(packed)
    vals = dict(zip(keys, packed.tolist()))
    n = max(vals.pop("num_samples"), 1.0)
    return {f"val/{k}": v / n for k, v in vals.items()}


def main(args) -> dict:
    info = pdist.init_distributed(args.device)
    set_trace_ranges(args.trace_ranges)
    device = info.device
    log = print if info.is_main else (lambda *a, **k: None)
    dtype = C.compute_dtype(args, device)
    model = build_model(args, device, dtype, info.rank)
    if args.pretrained_ckpt:
        tree = load_pretrained_params(args.pretrained_ckpt, model.flax_params(), log)
        model.store.load_flax_tree(tree, strict=False)
        log(f"Pretrained weights are loaded from {args.pretrained_ckpt}.")
    pdist.broadcast_(model.store.master)
    model.store.sync_shadow()
    C.summarize_params(model.store, log)
    if model.cfg.batch_norm:
        log("BatchNorm statistics are initialized.")
    peak = args.learning_rate * args.train_batch_size / 256 if args.optimizer == "lars" else args.learning_rate
    opt = C.make_optimizer(args, model.store, peak, 1e-6)
    reducer = C.make_reducer(args, model.store)
    rngs = RngStreams({"mixup": args.mixup_seed, "dropout": args.dropout_seed, "noise": args.noise_seed},
                      info.rank, device)
    trainer = Trainer(model, opt, reducer, rngs, args.grad_accum, skip_nonfinite=args.skip_nonfinite)
    run_step = StepRunner(trainer, hip_graph=args.hip_graph and device.type == "cuda" and info.world_size == 1)
    resumed = C.maybe_resume(args, model, opt, rngs, log)
    start = resumed.step

    def extra():
        if not model.cfg.batch_norm:
            return None
        return {"batch_stats": {"mean": model.head.running_mean.cpu(), "var": model.head.running_var.cpu()}}

    # a resumed run continues the data stream after the batches the interrupted run consumed
    train_loader, valid_loader = create_dataloaders(args, info.rank, info.world_size, resumed.batches,
                                                    device_augment=C.use_device_augment(args, device))
    result = {}
    logger = Logger(args.output_dir, args.name, args.project, vars(args), enabled=info.is_main,
                    use_wandb=False if args.log_file_only else None)
    if valid_loader is not None:  # SANITATION CHECK (main_finetune.py:53-54)
        result.update(evaluate(model, valid_loader, rngs, device))
        logger.log(dict(result), start)
        log(f"[eval] step {start} {result}")
    meter = AverageMeter(use_latest=["learning_rate"])
    max_acc1 = resumed.best("val/acc1", 0.0)
    it = C.DevicePrefetcher(train_loader, device) if train_loader is not None else None
    t0 = time.time()
    perf = C.PerfClock(start, args.train_batch_size, finetune_fwd_flops_per_image(model.cfg), info.world_size)
    step = start
    for step in range(start + 1, args.training_steps + 1):
        micro = [tuple(next(it)) for _ in range(args.grad_accum)]
        metrics = run_step(micro)
        meter.update(**metrics)
        if args.log_interval > 0 and step % args.log_interval == 0:
            summ = meter.summary("train/")
            summ["processed_samples"] = step * args.train_batch_size
            summ.update(perf.summary(step))
            comm = trainer.comm_ms()
            if comm is not None:
                summ["perf/comm_ms"] = comm
            C.check_finite(summ, step)
            if info.is_main:
                logger.log(summ, step)
                log(f"[train] step {step} " + " ".join(f"{k}={v:.5g}" for k, v in summ.items()))
        do_eval = args.eval_interval > 0 and (step % args.eval_interval == 0 or step == args.training_steps)
        stop = C.stop_here(args, step, start)
        do_save = do_eval or stop or (args.save_interval > 0 and step % args.save_interval == 0)
        # every rank's random state (collective), then rank 0 writes; "last" is written after the
        # evaluation so that its sidecar carries the updated best metric
        per_rank = C.rank_states(rngs, model) if do_save else None
        if do_eval and valid_loader is not None:
            res = evaluate(model, valid_loader, rngs, device)
            if res["val/acc1"] > max_acc1:  # identical on every rank (all-reduced)
                max_acc1 = res["val/acc1"]
                C.save_last(args, model, opt, step, rngs, extra(), postfix="best", per_rank=per_rank,
                            best={"val/acc1": max_acc1})
            if info.is_main:
                res["val/acc1/best"] = max_acc1
                res["processed_samples"] = step * args.train_batch_size
                logger.log(res, step)
                log(f"[eval] step {step} {res}")
            result.update(res)
        if do_save:
            C.save_last(args, model, opt, step, rngs, extra(), per_rank=per_rank, best={"val/acc1": max_acc1})
        if stop:
            log(f"[train] --stop-after-steps: stopping at step {step}")
            break
    C.flush_checkpoints()
    result["train_time_s"] = time.time() - t0
    result["final_step"] = step
    logger.close()
    return result


def cli(argv=None):
    args = finetune_parser().parse_args(argv)
    out = main(args)
    pdist.cleanup()
    return out


if __name__ == "__main__":
    cli()
