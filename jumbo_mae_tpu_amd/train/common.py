"""Pieces shared by the pretrain and finetune drivers."""

from __future__ import annotations

import os
import time

import torch

from ..ckpt.checkpoint import ckpt_path, load_params, load_resume_state, save_params, save_resume_state, writer
from ..optim.flat import FlatOptimizer
from ..optim.schedule import warmup_cosine_decay_schedule
from ..parallel import dist as pdist
from ..parallel.ddp import GradReducer


def pick_device(args) -> torch.device:
    return pdist.info().device


def compute_dtype(args, device) -> torch.dtype:
    if args.compute_dtype == "fp32" or (args.compute_dtype == "auto" and device.type != "cuda"):
        return torch.float32
    return torch.bfloat16


def summarize_params(store, log=print):
    """module.tabulate equivalent (pretraining.py:214): per-subtree parameter counts."""
    groups: dict[str, int] = {}
    for s in store.segments:
        key = "/".join(s.path[:2]) if s.path[0] == "model" else s.path[0]
        groups[key] = groups.get(key, 0) + s.numel
    width = max(len(k) for k in groups) + 2
    lines = [f"{'subtree'.ljust(width)}params"] + [f"{k.ljust(width)}{v:,}" for k, v in groups.items()]
    lines.append(f"{'TOTAL'.ljust(width)}{store.num_params():,} (trainable {store.num_params(True):,})")
    log("\n".join(lines))


def make_optimizer(args, store, peak_lr: float, end_value: float) -> FlatOptimizer:
    log = print if pdist.info().is_main else (lambda *a, **k: None)
    log(f"Peak learning rate: {peak_lr:.1e}")
    sched = warmup_cosine_decay_schedule(1e-6, peak_lr, args.warmup_steps, args.training_steps, end_value)
    return FlatOptimizer(store, args.optimizer, sched, b1=args.adam_b1, b2=args.adam_b2, eps=args.adam_eps,
                         weight_decay=args.weight_decay, lr_decay=args.lr_decay, num_layers=args.layers,
                         clip_grad=args.clip_grad)


def make_reducer(args, store):
    if pdist.info().world_size > 1:
        return GradReducer(store, bucket_mb=args.bucket_mb)
    return None


class DevicePrefetcher:
    """Moves the next host batch to the device on a side stream while the current step runs."""

    def __init__(self, it, device):
        self.it = iter(it)
        self.device = device
        self.stream = torch.cuda.Stream(device) if device.type == "cuda" else None
        self.next = None
        self._preload()

    def _to(self, b):
        if isinstance(b, (list, tuple)):
            return type(b)(self._to(x) for x in b)
        if isinstance(b, torch.Tensor):
            return b.to(self.device, non_blocking=True)
        return b

    def _preload(self):
        try:
            b = next(self.it)
        except StopIteration:
            self.next = None
            return
        if self.stream is not None:
            with torch.cuda.stream(self.stream):
                self.next = self._to(b)
        else:
            self.next = self._to(b)

    def __iter__(self):
        return self

    def __next__(self):
        if self.next is None:
            raise StopIteration
        if self.stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
            for t in (self.next if isinstance(self.next, (list, tuple)) else [self.next]):
                if isinstance(t, torch.Tensor):
                    t.record_stream(torch.cuda.current_stream(self.device))
        b = self.next
        self._preload()
        return b


def save_last(args, model, opt, step, rngs, extra_state=None, postfix="last"):
    """Rank 0: params msgpack (Flax tree) + resume sidecar, both written in the background."""
    if not pdist.info().is_main:
        return None
    tree = model.flax_params()
    if hasattr(model, "batch_stats") and model.batch_stats() is not None:
        pass  # batch_stats live in the sidecar (reference does not save them at all)
    url = save_params(args.output_dir, args.name or "run", tree, postfix)
    state = {"step": step, "optimizer": opt.state_dict(), "rngs": rngs.state_dict() if rngs else {},
             "time": time.time()}
    if extra_state:
        state.update(extra_state)
    save_resume_state(ckpt_path(args.output_dir, args.name or "run", postfix, "state.pt"), state)
    return url


def maybe_resume(args, model, opt, rngs, log=print):
    """--resume auto|<prefix>: restore params, optimizer moments/count, RNG streams; returns step."""
    if not args.resume:
        return 0
    prefix = os.path.join(args.output_dir, f"{args.name or 'run'}-last") if args.resume == "auto" else args.resume
    pfile, sfile = prefix + ".msgpack", prefix + ".state.pt"
    if not (os.path.exists(pfile) and os.path.exists(sfile)):
        log(f"[resume] nothing to resume at {prefix}")
        return 0
    model.store.load_flax_tree(load_params(pfile), strict=True)
    st = load_resume_state(sfile)
    opt.load_state_dict(st["optimizer"])
    if rngs is not None and st.get("rngs"):
        rngs.load_state_dict(st["rngs"])
    if "batch_stats" in st and hasattr(model, "head") and getattr(model.head, "running_mean", None) is not None:
        model.head.running_mean.copy_(st["batch_stats"]["mean"])
        model.head.running_var.copy_(st["batch_stats"]["var"])
    pdist.broadcast_(model.store.master)
    model.store.sync_shadow()
    log(f"[resume] restored step {st['step']} from {prefix}")
    return int(st["step"])


def flush_checkpoints():
    writer().flush()


def check_finite(metrics: dict, step: int):
    """Non-finite loss detection: abort with a clear message."""
    v = metrics.get("train/loss")
    if v is not None and not (v == v and abs(v) != float("inf")):
        raise FloatingPointError(f"non-finite training loss at step {step}: {v}")


class PerfClock:
    """perf/* log keys: images/sec, step time and MFU over each log window."""

    def __init__(self, start_step: int, global_batch: int, fwd_flops_per_image: float, world_size: int):
        self.t, self.step = time.time(), start_step
        self.batch, self.flops, self.world = global_batch, fwd_flops_per_image, world_size

    def summary(self, step: int) -> dict:
        from ..utils.flops import mfu
        now = time.time()
        dt = max(now - self.t, 1e-9)
        n = max(step - self.step, 1)
        ips = n * self.batch / dt
        self.t, self.step = now, step
        return {"perf/images_per_sec": ips, "perf/step_ms": 1e3 * dt / n,
                "perf/mfu": mfu(ips, self.flops, self.world)}
