"""Pieces shared by the pretrain and finetune drivers."""

from __future__ import annotations

import time

import torch

from ..ckpt.checkpoint import ckpt_path, load_params, load_resume_state, save_params, save_resume_state, writer
from ..optim.flat import FlatOptimizer
from ..optim.schedule import warmup_cosine_decay_schedule
from ..parallel import dist as pdist
from ..parallel.ddp import GradReducer
from ..utils import gopen


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
    if pdist.info().world_size > 1 or pdist.forced_group():
        dt = torch.bfloat16 if getattr(args, "reduce_dtype", "fp32") == "bf16" else torch.float32
        return GradReducer(store, bucket_mb=args.bucket_mb, reduce_dtype=dt,
                           shard=getattr(args, "shard_optimizer", False),
                           gather_dtype=getattr(args, "zero1_gather", "bf16"))
    return None


def use_device_augment(args, device) -> bool:
    """--device-augment: auto = on a GPU with the extension and the pretraining train transform."""
    from ..data.loader import device_augment_ok
    mode = getattr(args, "device_augment", "off")
    if mode == "off" or device.type != "cuda" or not getattr(args, "train_dataset_shards", None):
        return False
    if not device_augment_ok(args):
        if mode == "on":
            raise SystemExit("--device-augment on: the train transform must be RandomResizedCrop + flip only")
        return False
    from ..ops import _ext
    if not _ext.available():  # no built extension (JMAE_ALLOW_TORCH_FALLBACK runs): the PIL path
        if mode == "on":
            raise SystemExit("--device-augment on needs the built HIP extension (python -m jumbo_mae_tpu_amd.csrc.build)")
        return False
    return True


class DevicePrefetcher:
    """Moves the next host batch to the device on a side stream while the current step runs; a
    device-augment batch (data/loader.py ``PackedImages``) is resized / flipped there too."""

    def __init__(self, it, device):
        self.it = iter(it)
        self.device = device
        self.stream = torch.cuda.Stream(device) if device.type == "cuda" else None
        self.next = None
        self._preload()

    def _to(self, b):
        from ..data.loader import PackedImages, unpack_on_device
        if isinstance(b, PackedImages):
            return unpack_on_device(b, self.device)
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


def rank_states(rngs, model) -> list:
    """COLLECTIVE (every rank calls it at the same step): each rank's random state -- its device
    streams (mixup / dropout / noise) and the host Mixup generator -- gathered in rank order.
    Saved in the resume sidecar so that after ``--resume`` every rank continues its OWN streams
    (the reference's per-device ``shard_prng_key`` independence), not rank 0's."""
    mine = {"rngs": rngs.state_dict() if rngs is not None else {}}
    mix = getattr(model, "mixup", None)
    if mix is not None and getattr(mix, "rs", None) is not None:
        mine["mixup_host"] = mix.rs.bit_generator.state
    return pdist.all_gather_object(mine)


def save_last(args, model, opt, step, rngs, extra_state=None, postfix="last", per_rank=None, best=None):
    """Rank 0: params msgpack (Flax tree) + resume sidecar, both written in the background.

    The sidecar holds the optimizer state, every rank's random state (``per_rank`` from
    ``rank_states``), the data position (train batches consumed per rank) and the best
    validation metric so far."""
    if hasattr(opt, "gather_state"):
        opt.gather_state()  # collective: sharded optimizer moments made whole on every rank
    if not pdist.info().is_main:
        return None
    tree = model.flax_params()
    url = save_params(args.output_dir, args.name or "run", tree, postfix)
    state = {"step": step, "optimizer": opt.state_dict(), "rngs": rngs.state_dict() if rngs else {},
             "time": time.time(), "world_size": pdist.info().world_size,
             "data": {"batches_per_rank": step * getattr(args, "grad_accum", 1)}}
    if per_rank is not None:
        state["rngs_per_rank"] = per_rank
    if best is not None:
        state["best"] = dict(best)
    if extra_state:
        state.update(extra_state)
    save_resume_state(ckpt_path(args.output_dir, args.name or "run", postfix, "state.pt"), state)
    return url


class Resumed(dict):
    """What ``maybe_resume`` restored: step, data position and best metrics (empty = fresh run)."""

    @property
    def step(self) -> int:
        return int(self.get("step", 0))

    @property
    def batches(self) -> int:
        return int(self.get("data", {}).get("batches_per_rank", 0))

    def best(self, key: str, default: float) -> float:
        return float(self.get("best", {}).get(key, default))


def maybe_resume(args, model, opt, rngs, log=print) -> Resumed:
    """--resume auto|<prefix>: restore params, optimizer moments/count, this rank's RNG streams and
    host Mixup generator; returns the step, data position and best metrics (``Resumed``)."""
    if not args.resume:
        return Resumed()
    prefix = gopen.join(args.output_dir, f"{args.name or 'run'}-last") if args.resume == "auto" else args.resume
    pfile, sfile = prefix + ".msgpack", prefix + ".state.pt"
    if not (gopen.exists(pfile) and gopen.exists(sfile)):
        log(f"[resume] nothing to resume at {prefix}")
        return Resumed()
    model.store.load_flax_tree(load_params(pfile), strict=True)
    st = load_resume_state(sfile)
    opt.load_state_dict(st["optimizer"])
    info = pdist.info()
    per_rank = st.get("rngs_per_rank")
    if per_rank is not None and len(per_rank) == info.world_size:
        mine = per_rank[info.rank]
        if rngs is not None and mine.get("rngs"):
            rngs.load_state_dict(mine["rngs"])
        mix = getattr(model, "mixup", None)
        if mine.get("mixup_host") is not None and mix is not None and getattr(mix, "rs", None) is not None:
            mix.rs.bit_generator.state = mine["mixup_host"]
    elif rngs is not None:
        # saved with another world size (or by an older version): fresh per-rank streams keyed by
        # the step, so ranks stay independent and do not replay the first steps' draws
        rngs.reseed(int(st["step"]))
        log("[resume] world size changed or no per-rank RNG state: streams re-derived from (seed, rank, step)")
    if "batch_stats" in st and hasattr(model, "head") and getattr(model.head, "running_mean", None) is not None:
        model.head.running_mean.copy_(st["batch_stats"]["mean"])
        model.head.running_var.copy_(st["batch_stats"]["var"])
    pdist.broadcast_(model.store.master)
    model.store.sync_shadow()
    log(f"[resume] restored step {st['step']} from {prefix}")
    out = Resumed(step=int(st["step"]), best=st.get("best", {}))
    if "data" in st and st.get("world_size", info.world_size) == info.world_size:
        out["data"] = st["data"]
    return out


def stop_here(args, step: int, start: int) -> bool:
    """--stop-after-steps: this invocation has run its share of steps."""
    n = getattr(args, "stop_after_steps", 0)
    return n > 0 and step - start >= n and step < args.training_steps


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
