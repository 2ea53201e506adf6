"""MAE pretraining driver (``main_pretrain``).

Parity: /root/reference/src/main_pretrain.py:37-94 and create_train_state
(/root/reference/src/pretraining.py:170-270):
  * peak LR = learning_rate * train_batch_size / 256, warmup-cosine from 1e-6 to 1e-5;
  * "SANITATION CHECK" validation before training (skipped when there is no validation set, Q8);
  * metrics averaged over log_interval with the latest learning_rate, keys train/loss,
    train/learning_rate, processed_samples, val/loss, val/loss/best;
  * at eval_interval (and the last step): evaluates, saves ``{name}-best.msgpack`` on a new minimum
    validation loss and ``{name}-last.msgpack`` (the reference writes "last" before the evaluation;
    here it follows it so that its resume sidecar carries the updated best metric).
Launch: ``torchrun --nproc-per-node 8 src/main_pretrain.py <reference flags>``.
"""

from __future__ import annotations

import time

import torch

from ..config import DecoderConfig, ViTConfig
from ..data.loader import create_dataloaders
from ..models.mae import PretrainModel
from ..parallel import dist as pdist
from ..utils.flops import pretrain_fwd_flops_per_image
from ..utils.rng import RngStreams
from ..utils.trace import set_enabled as set_trace_ranges
from . import common as C
from .cli import pretrain_parser
from ..runtime.graph import StepRunner
from .engine import Trainer
from .meter import AverageMeter, Logger


def build_model(args, device, dtype) -> PretrainModel:
    vc = ViTConfig(layers=args.layers, dim=args.dim, heads=args.heads, labels=args.labels, layerscale=args.layerscale,
                   patch_size=args.patch_size, image_size=args.image_size, posemb=args.posemb, pooling=args.pooling,
                   dropout=args.dropout, droppath=args.droppath, grad_ckpt=args.grad_ckpt,
                   image_mask_ratio=args.image_mask_ratio, linear_probing=False)
    dc = DecoderConfig(dec_layers=args.dec_layers, dec_dim=args.dec_dim, dec_heads=args.dec_heads,
                       dec_layerscale=args.dec_layerscale, dec_posemb=args.dec_posemb, dec_dropout=args.dec_dropout,
                       dec_droppath=args.dec_droppath, grad_ckpt=args.grad_ckpt, patch_size=args.patch_size,
                       image_size=args.image_size)
    return PretrainModel(vc, dc, norm_pix_loss=args.norm_pix_loss,
                         mask_mode=getattr(args, "mask_mode", "shared")).to(device, dtype, seed=args.init_seed)


def evaluate(model, loader, rngs, device) -> dict:
    rngs = rngs.fork()  # validation never advances the training streams
    sums = None
    for batch in C.DevicePrefetcher(loader, device):
        images, labels = batch if isinstance(batch, (list, tuple)) else (batch, None)
        valid = (labels != -1) if labels is not None else None
        m = model.evaluate(images, valid, rngs.as_dict())
        sums = m if sums is None else {k: sums[k] + m[k] for k in m}
    packed = torch.stack([sums["loss"], sums["num_samples"]]).float()
    pdist.all_reduce_sum_(packed)
    loss, n = packed.tolist()
    return {"val/loss": loss / max(n, 1.0)}


def main(args) -> dict:
    info = pdist.init_distributed(args.device)
    set_trace_ranges(args.trace_ranges)
    device = info.device
    log = print if info.is_main else (lambda *a, **k: None)
    dtype = C.compute_dtype(args, device)
    model = build_model(args, device, dtype)
    pdist.broadcast_(model.store.master)  # CC6: identical initial params on every rank
    model.store.sync_shadow()
    C.summarize_params(model.store, log)
    opt = C.make_optimizer(args, model.store, args.learning_rate * args.train_batch_size / 256, 1e-5)
    reducer = C.make_reducer(args, model.store)
    rngs = RngStreams({"mixup": args.mixup_seed, "dropout": args.dropout_seed, "noise": args.noise_seed},
                      info.rank, device)
    trainer = Trainer(model, opt, reducer, rngs, args.grad_accum, skip_nonfinite=args.skip_nonfinite)
    run_step = StepRunner(trainer, hip_graph=args.hip_graph and device.type == "cuda" and info.world_size == 1)
    resumed = C.maybe_resume(args, model, opt, rngs, log)
    start = resumed.step

    # a resumed run continues the data stream after the batches the interrupted run consumed
    train_loader, valid_loader = create_dataloaders(args, info.rank, info.world_size, resumed.batches,
                                                    device_augment=C.use_device_augment(args, device))
    result = {}
    logger = Logger(args.output_dir, args.name, args.project, vars(args), enabled=info.is_main,
                    use_wandb=False if args.log_file_only else None)
    if valid_loader is not None:  # SANITATION CHECK (main_pretrain.py:53-54), skipped without a valid set (Q8)
        result.update(evaluate(model, valid_loader, rngs, device))
        logger.log(dict(result), start)
        log(f"[eval] step {start} {result}")
    meter = AverageMeter(use_latest=["learning_rate"])
    min_val_loss = resumed.best("val/loss", 1e9)
    it = C.DevicePrefetcher(train_loader, device) if train_loader is not None else None
    t0 = time.time()
    perf = C.PerfClock(start, args.train_batch_size, pretrain_fwd_flops_per_image(model.cfg, model.dec_cfg),
                       info.world_size)
    step = start
    for step in range(start + 1, args.training_steps + 1):
        micro = []
        for _ in range(args.grad_accum):
            b = next(it)
            micro.append((b[0] if isinstance(b, (list, tuple)) else b,))
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
            if res["val/loss"] < min_val_loss:  # identical on every rank (all-reduced)
                min_val_loss = res["val/loss"]
                C.save_last(args, model, opt, step, rngs, postfix="best", per_rank=per_rank,
                            best={"val/loss": min_val_loss})
            if info.is_main:
                res["val/loss/best"] = min_val_loss
                res["processed_samples"] = step * args.train_batch_size
                logger.log(res, step)
                log(f"[eval] step {step} {res}")
            result.update(res)
        if do_save:
            C.save_last(args, model, opt, step, rngs, per_rank=per_rank, best={"val/loss": min_val_loss})
        if stop:
            log(f"[train] --stop-after-steps: stopping at step {step}")
            break
    C.flush_checkpoints()
    result["train_time_s"] = time.time() - t0
    result["final_step"] = step
    logger.close()
    return result


def cli(argv=None):
    args = pretrain_parser().parse_args(argv)
    out = main(args)
    pdist.cleanup()
    return out


if __name__ == "__main__":
    cli()
