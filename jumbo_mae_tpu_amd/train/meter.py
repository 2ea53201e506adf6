"""Metric buffering and logging.

Reference: ``AverageMeter`` (/root/reference/src/utils.py:36-52) -- buffers every micro-step's
metrics (device arrays, no sync) and summarizes at ``log_interval`` (mean, or latest value for
keys in ``use_latest`` such as ``learning_rate``) -- and wandb logging on process 0
(main_pretrain.py:56-57,67-74).  wandb is not installed offline, so the default sink is a JSONL
file with the same keys; a wandb sink is used when the package is importable and requested.
Device tensors are stacked and reduced over ranks in ONE packed all-reduce per summary (the
reference pmean's every step).
"""

from __future__ import annotations

import json
import os
import time
from collections import defaultdict

import numpy as np
import torch
import torch.distributed as dist

from ..utils import gopen


class AverageMeter:
    def __init__(self, use_latest: list[str] | None = None, group=None):
        self.buffer = defaultdict(list)
        self.use_latest = list(use_latest or [])
        self.group = group

    def update(self, **kwargs):
        for k, v in kwargs.items():
            self.buffer[k].append(v)

    def summary(self, prefix: str = "", reduce: bool = True) -> dict[str, float]:
        keys = list(self.buffer.keys())
        vals = []
        for k in keys:
            v = self.buffer[k]
            if k in self.use_latest:
                x = v[-1]
                x = x.detach().float().mean() if isinstance(x, torch.Tensor) else torch.tensor(float(x))
            else:
                if isinstance(v[0], torch.Tensor):
                    x = torch.stack([t.detach().float().reshape(()) for t in v]).mean()
                else:
                    x = torch.tensor(float(np.mean(v)))
            vals.append(x)
        self.buffer.clear()
        if not keys:
            return {}
        dev = next((t.device for t in vals if t.device.type != "cpu"), torch.device("cpu"))
        packed = torch.stack([t.to(dev) for t in vals])
        if reduce and dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1:
            dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=self.group)
            packed = packed / dist.get_world_size(self.group)  # pmean (latest values agree on all ranks)
        out = packed.cpu().tolist()
        return {f"{prefix}{k}": float(v) for k, v in zip(keys, out)}


class Logger:
    """JSONL metrics sink (+ optional wandb) for rank 0."""

    def __init__(self, output_dir: str, name: str | None, project: str | None = None, config: dict | None = None,
                 enabled: bool = True, use_wandb: bool | None = None):
        self.enabled = enabled
        self.f = None
        self.wandb = None
        if not enabled:
            return
        # a remote --output-dir (gs://...) keeps the metrics log in the working directory
        log_dir = output_dir or "."
        if not gopen.is_local(log_dir):
            log_dir = "."
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, f"{name or 'run'}-metrics.jsonl")
        self.f = open(self.path, "a")
        if use_wandb is None:
            use_wandb = os.environ.get("WANDB_MODE", "") not in ("", "disabled") or bool(os.environ.get("WANDB_API_KEY"))
        if use_wandb:
            try:
                import wandb  # noqa: F401
                self.wandb = wandb
                wandb.init(name=name, project=project, config=config)
            except Exception:
                self.wandb = None
        self.log({"config": config or {}}, step=0)

    def log(self, metrics: dict, step: int):
        if not self.enabled:
            return
        rec = {"step": step, "time": time.time(), **metrics}
        self.f.write(json.dumps(rec, default=float) + "\n")
        self.f.flush()
        if self.wandb is not None and "config" not in metrics:
            self.wandb.log(metrics, step)

    def close(self):
        if self.f:
            self.f.close()
