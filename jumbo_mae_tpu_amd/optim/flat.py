"""Fused optimizers over the flat parameter store, with optax semantics.

Parity (reference):
  adamw  = optax.adamw(lr, b1, b2, eps, weight_decay, mask=kernel)      pretraining.py:223-233
  lamb   = modified_lamb: scale_by_adam -> add_decayed_weights(mask) ->
           masked(scale_by_trust_ratio, mask) -> scale_by_lr            utils.py:124-139
  lars   = optax.lars(lr, momentum=0.9): add_decayed_weights(0) ->
           scale_by_trust_ratio(0.001) -> scale_by_lr -> trace(0.9)      finetuning.py:230-234
  sgd    = optax.sgd(lr, momentum=0.9): trace(0.9) -> scale_by_lr       finetuning.py:225-229
  LLRD   = chain(tx, multi_transform(scale(lr_decay**(L-i)), label))   pretraining.py:234-241
  clip   = chain(clip_by_global_norm(c), tx)                            pretraining.py:242-243
  LR     = inject_hyperparams(schedule)(count), count from 0            pretraining.py:221-259

Execution: on the GPU every optimizer is ONE fused pass over the flat fp32 master / grad /
moment buffers driven by a chunk table (multi-tensor apply), which also rewrites the bf16
shadow weights; LAMB/LARS add one per-segment norm pass (trust ratios are per Flax leaf,
exactly like optax on the reference tree).  Per-step scalars (lr, bias corrections, clip
factor) live in a small device tensor so the step is HIP-graph capturable.  The torch path
(CPU) implements the same math with per-element metadata vectors.
"""

from __future__ import annotations

import re

import torch

from ..models.params import ParamStore
from ..ops import _ext
from .schedule import WarmupCosine

# elements per chunk of the multi-tensor table: one workgroup each; 8 Ki elements keep more
# workgroups in flight than 64 Ki (AdamW alone: 551 -> 493 us at 86 M parameters, 2383 -> 2303 us
# at 400 M, tools/adamw_bench.py --chunk, profiles/r4zb_adamw_chunk.txt)
CHUNK = 8192


def layer_index(path: tuple[str, ...], num_layers: int) -> int:
    """get_layer_index_fn (/root/reference/src/utils.py:142-147)."""
    if path[0] == "model" and len(path) > 1 and path[1].startswith("layer_"):
        return int(re.match(r"layer_(\d+)", path[1]).group(1)) + 1
    if path[0] == "model" and len(path) > 1 and path[1] == "embed":
        return 0
    return num_layers


class FlatOptimizer:
    KINDS = ("adamw", "lamb", "lars", "sgd")

    def __init__(self, store: ParamStore, kind: str, schedule: WarmupCosine, *, b1=0.9, b2=0.999,
                 eps=1e-8, weight_decay=0.0, lr_decay=1.0, num_layers=12, clip_grad=0.0,
                 momentum=0.9, trust_coefficient=0.001):
        assert kind in self.KINDS, kind
        self.store, self.kind, self.schedule = store, kind, schedule
        self.b1, self.b2, self.eps = b1, b2, eps
        self.weight_decay = weight_decay if kind in ("adamw", "lamb") else 0.0
        self.lr_decay, self.num_layers = lr_decay, num_layers
        self.clip_grad = clip_grad
        self.momentum, self.trust_coefficient = momentum, trust_coefficient
        self.count = 0  # optax inject_hyperparams count (host mirror)
        self.last_lr = schedule(0)
        dev = store.master.device
        n = store.total
        segs = store.segments
        self.nseg = len(segs)
        # ---- per-segment metadata: [decay flag, llrd scale, trust flag]
        meta = torch.zeros(self.nseg, 4, dtype=torch.float32)
        for i, s in enumerate(segs):
            decay = 1.0 if (s.is_kernel and self.weight_decay > 0) else 0.0
            llrd = lr_decay ** (num_layers - layer_index(s.path, num_layers)) if lr_decay < 1.0 else 1.0
            trust = 1.0 if (kind == "lars" or (kind == "lamb" and s.is_kernel)) else 0.0
            meta[i] = torch.tensor([decay, llrd, trust, 1.0 if s.trainable else 0.0])
        self.meta = meta.to(dev)
        # ---- chunk table for the multi-tensor kernels: [start, length, segment]
        rows = []
        for i, s in enumerate(segs):
            for st in range(0, s.numel, CHUNK):
                rows.append((s.offset + st, min(CHUNK, s.numel - st), i))
        self.chunks = torch.tensor(rows, dtype=torch.int64).to(torch.int32).to(dev)
        # ---- state
        self.mu = torch.zeros(n, dtype=torch.float32, device=dev) if kind in ("adamw", "lamb") else None
        self.nu = torch.zeros(n, dtype=torch.float32, device=dev) if kind in ("adamw", "lamb") else None
        self.trace = torch.zeros(n, dtype=torch.float32, device=dev) if kind in ("lars", "sgd") else None
        self.hyper = torch.zeros(8, dtype=torch.float32, device=dev)
        self.norms = torch.zeros(self.nseg, 2, dtype=torch.float32, device=dev)
        self.gnorm_sq = torch.zeros(1, dtype=torch.float32, device=dev)
        self._tmp = None
        self._torch_meta = None
        self._ranges = None      # (lo, hi) -> chunk-table rows (split updates, plan_ranges)
        self._rest = None        # chunk-table rows outside every planned range
        self._gn_ready = False   # gnorm_sq flag written for this step (split updates)
        self._shard = None       # GradReducer in ZeRO-1 mode: update only this rank's pieces
        self._owned_rows = None  # chunk-table rows of every owned piece
        self._owned_mask = None  # torch path: bool mask of owned elements

    # ---------------------------------------------------------------- helpers
    def _elem_meta(self):
        """Per-element metadata for the torch path (built lazily)."""
        if self._torch_meta is None:
            s = self.store
            seg_id = torch.zeros(s.total, dtype=torch.int64, device=s.master.device)
            valid = torch.zeros(s.total, dtype=torch.bool, device=s.master.device)
            for i, seg in enumerate(s.segments):
                seg_id[seg.offset:seg.offset + seg.numel] = i
                valid[seg.offset:seg.offset + seg.numel] = True
            m = self.meta[seg_id]
            self._torch_meta = (seg_id, valid, m[:, 0], m[:, 1], m[:, 2] > 0, m[:, 3] > 0)
        return self._torch_meta

    def _seg_norm_sq(self, x: torch.Tensor, seg_id: torch.Tensor, valid: torch.Tensor) -> torch.Tensor:
        out = torch.zeros(self.nseg, dtype=torch.float32, device=x.device)
        out.index_add_(0, seg_id[valid], (x[valid] * x[valid]))
        if self._shard is not None:
            self._shard.sum_(out)
        return out

    # ---------------------------------------------------------------- step
    def step(self) -> float:
        """Apply one optimizer update from ``store.grad``; returns the learning rate used."""
        self.prepare()
        self.launch()
        return self.finish()

    # A step in three parts so the device work can be captured in a HIP graph
    # (runtime/graph.py): ``prepare`` (host: schedule value, bias corrections -> the static
    # ``hyper`` device buffer through the step feeder), ``launch`` (device kernels only),
    # ``finish`` (host bookkeeping).
    def prepare(self) -> None:
        lr = float(self.schedule(self.count))
        t = self.count + 1
        self._cur = (lr, 1.0 - self.b1 ** t, 1.0 - self.b2 ** t)
        s = self.store
        if s.master.is_cuda and _ext.use_hip(s.master):
            from ..runtime.feeder import feeder
            lr, bc1, bc2 = self._cur
            # hyper = [lr, bc1, bc2, clip, b1, b2, eps, wd]
            self.hyper = feeder(s.master.device).put(
                "opt_hyper", [lr, bc1, bc2, self.clip_grad, self.b1, self.b2, self.eps, self.weight_decay])

    def launch(self) -> None:
        s = self.store
        if s.master.is_cuda and _ext.use_hip(s.master):
            self._step_hip()
        else:
            self._step_torch(*self._cur)

    # Split updates: the elementwise optimizers (AdamW, SGD without global-norm clipping) update
    # each data-parallel bucket as soon as its all-reduce has completed (GradReducer.finish
    # callback), so the update of the early buckets overlaps the reduction of the last ones.
    def can_split(self) -> bool:
        return self.kind in ("adamw", "sgd") and self.clip_grad <= 0

    def attach_shard(self, reducer) -> None:
        """ZeRO-1: from now on every update touches only ``reducer``'s owned pieces (the rest of the
        master arrives by the reducer's all-gather); norms and the clip norm are summed over ranks."""
        if reducer is None or not getattr(reducer, "shard", False):
            return
        self._shard = reducer
        pieces = reducer.owned_pieces()
        self._owned_rows = self._rows_for(pieces)
        own = torch.zeros(self.store.total, dtype=torch.bool, device=self.store.master.device)
        for a, b in pieces:
            own[a:b] = True
        self._owned_mask = own

    def _rows_for(self, pieces: list[tuple[int, int]]):
        """Chunk-table rows covering exactly the segment elements inside ``pieces``."""
        rows = []
        for a, b in sorted(pieces):
            for i, sg in enumerate(self.store.segments):
                lo, hi = max(a, sg.offset), min(b, sg.offset + sg.numel)
                for st in range(lo, hi, CHUNK):
                    rows.append((st, min(CHUNK, hi - st), i))
        if not rows:
            return None
        return torch.tensor(rows, dtype=torch.int64).to(torch.int32).to(self.store.master.device)

    def gather_state(self) -> None:
        """COLLECTIVE (every rank, same step): make the sharded moments whole on every rank before
        ``state_dict`` (checkpoint).  No-op without sharding."""
        if self._shard is not None:
            self._shard.gather_state([self.mu, self.nu, self.trace])

    def plan_ranges(self, ranges: list[tuple[int, int]], pieces: list[list[tuple[int, int]]] | None = None) -> None:
        """Rows of each split-update range.  ``pieces`` (sharded): the exact element ranges of each
        range that this rank updates; nothing outside them is ever updated."""
        if pieces is not None:
            self._ranges = {r: self._rows_for(pc) for r, pc in zip(ranges, pieces)}
            self._rest = None
            return
        starts = self.chunks[:, 0].long().cpu()
        covered = torch.zeros(len(starts), dtype=torch.bool)
        self._ranges = {}
        for lo, hi in ranges:
            m = (starts >= lo) & (starts < hi)
            covered |= m
            self._ranges[(lo, hi)] = self._rows(m)
        self._rest = self._rows(~covered)

    def _rows(self, mask: torch.Tensor):
        idx = torch.nonzero(mask).flatten()
        if idx.numel() == 0:
            return None
        if int(idx[-1]) - int(idx[0]) + 1 == idx.numel():  # contiguous rows: a view
            return self.chunks[int(idx[0]):int(idx[-1]) + 1]
        return self.chunks.index_select(0, idx.to(self.chunks.device))

    def launch_range(self, lo: int, hi: int) -> None:
        """Update the parameters of flat range [lo, hi) (a planned bucket)."""
        rows = self._ranges[(lo, hi)]
        if rows is not None:
            self._launch_rows(rows, lo, hi)

    def launch_rest(self) -> None:
        """Update everything no planned range covers; ends a split step."""
        if self._rest is not None and self._shard is None:
            self._launch_rows(self._rest, None, None)
        self._gn_ready = False

    def _launch_rows(self, rows, lo, hi) -> None:
        s = self.store
        if s.master.is_cuda and _ext.use_hip(s.master):
            ext = _ext.load()
            if not self._gn_ready:
                self.gnorm_sq.fill_(-1.0)  # no clipping on the split path
                self._gn_ready = True
            shadow = s.shadow if s.shadow is not s.master else None
            if self.kind == "adamw":
                ext.opt_adamw(s.master, s.grad, self.mu, self.nu, shadow, rows, self.meta, self.hyper, self.gnorm_sq)
            else:
                ext.opt_sgd(s.master, s.grad, self.trace, shadow, rows, self.meta, self.hyper, self.gnorm_sq,
                            self.momentum)
        else:
            for r0, n, _ in rows.tolist():
                self._step_torch(*self._cur, lo=r0, hi=r0 + n)

    def finish(self) -> float:
        lr = self._cur[0]
        self.count += 1
        self.store.version += 1  # shadow rewritten: transposed weight copies are stale
        self.last_lr = lr
        return lr

    def _clip_scale_torch(self, g: torch.Tensor) -> torch.Tensor:
        if self.clip_grad <= 0:
            return torch.ones((), device=g.device)
        sq = (g * g).sum().reshape(1)
        if self._shard is not None:
            self._shard.sum_(sq)
        gn = torch.sqrt(sq[0])
        return torch.where(gn < self.clip_grad, torch.ones_like(gn), self.clip_grad / gn)

    @torch.no_grad()
    def _step_torch(self, lr, bc1, bc2, lo: int | None = None, hi: int | None = None):
        s = self.store
        if lo is not None:  # elementwise optimizers on one chunk of the flat buffer (split step)
            sl = slice(lo, hi)
            seg_id, valid, decay, llrd, trust_m, trainable = (t[sl] for t in self._elem_meta())
            p, g = s.master[sl], s.grad[sl]
            if self.kind == "adamw":
                self.mu[sl].mul_(self.b1).add_((1 - self.b1) * g)
                self.nu[sl].mul_(self.b2).add_((1 - self.b2) * g * g)
                u = (self.mu[sl] / bc1) / (torch.sqrt(self.nu[sl] / bc2) + self.eps)
                upd = -lr * (u + self.weight_decay * decay * p) * llrd
            else:  # sgd
                self.trace[sl].mul_(self.momentum).add_(g)
                upd = -lr * self.trace[sl] * llrd
            p.add_(torch.where(trainable & valid, upd, torch.zeros_like(upd)))
            if s.shadow is not s.master:
                s.shadow[sl].copy_(p)
            return
        p, g = s.master, s.grad
        seg_id, valid, decay, llrd, trust_m, trainable = self._elem_meta()
        own = self._owned_mask
        if own is not None:  # ZeRO-1: norms over the owned elements, summed over the ranks
            valid = valid & own
        g = g * self._clip_scale_torch(torch.where(valid, g, torch.zeros_like(g)))  # segments only
        if own is not None:  # moments / traces of non-owned pieces are left alone
            g = torch.where(own, g, torch.zeros_like(g))
            saved = [t.clone() for t in (self.mu, self.nu, self.trace) if t is not None]
        if self.kind in ("adamw", "lamb"):
            self.mu.mul_(self.b1).add_((1 - self.b1) * g)
            self.nu.mul_(self.b2).add_((1 - self.b2) * g * g)
            u = (self.mu / bc1) / (torch.sqrt(self.nu / bc2) + self.eps)
            u = u + self.weight_decay * decay * p
            if self.kind == "lamb":
                pn = torch.sqrt(self._seg_norm_sq(p, seg_id, valid))
                un = torch.sqrt(self._seg_norm_sq(u, seg_id, valid))
                tr = pn / un
                tr = torch.where((pn == 0) | (un == 0), torch.ones_like(tr), tr)
                u = torch.where(trust_m, u * tr[seg_id], u)
            upd = -lr * u * llrd
        elif self.kind == "lars":
            u = g  # weight_decay 0 (reference passes none)
            pn = torch.sqrt(self._seg_norm_sq(p, seg_id, valid))
            un = torch.sqrt(self._seg_norm_sq(u, seg_id, valid))
            tr = self.trust_coefficient * pn / un
            tr = torch.where((pn == 0) | (un == 0), torch.ones_like(tr), tr)
            u = u * tr[seg_id]
            u = -lr * u
            self.trace.mul_(self.momentum).add_(u)
            upd = self.trace * llrd
        else:  # sgd
            self.trace.mul_(self.momentum).add_(g)
            upd = -lr * self.trace * llrd
        upd = torch.where(trainable & valid, upd, torch.zeros_like(upd))
        p.add_(upd)
        if own is not None:
            for t, old in zip([t for t in (self.mu, self.nu, self.trace) if t is not None], saved):
                t.copy_(torch.where(own, t, old))
            if s.shadow is not s.master:  # owned pieces only: the rest arrives by the all-gather
                s.shadow.copy_(torch.where(own, p, s.shadow.float()))
                return
        s.sync_shadow()

    @torch.no_grad()
    def _step_hip(self):
        ext = _ext.load()
        s = self.store
        shadow = s.shadow if s.shadow is not s.master else None
        rows = self.chunks
        red = self._shard
        if red is not None:  # ZeRO-1: this rank's pieces only; per-leaf / global norms summed over ranks
            rows = self._owned_rows
            if rows is None:
                return
        if self.clip_grad > 0:
            self.gnorm_sq.zero_()
            ext.opt_sumsq(s.grad, rows, self.gnorm_sq)
            if red is not None:
                red.sum_(self.gnorm_sq)
        else:
            self.gnorm_sq.fill_(-1.0)
        if self.kind == "adamw":
            ext.opt_adamw(s.master, s.grad, self.mu, self.nu, shadow, rows, self.meta,
                          self.hyper, self.gnorm_sq)
        elif self.kind == "lamb":
            if self._tmp is None:
                self._tmp = torch.empty_like(s.master)
            self.norms.zero_()
            ext.opt_lamb_phase1(s.master, s.grad, self.mu, self.nu, self._tmp, rows, self.meta,
                                self.hyper, self.gnorm_sq, self.norms)
            if red is not None:
                red.sum_(self.norms)
            ext.opt_apply_trust(s.master, self._tmp, None, shadow, rows, self.meta, self.hyper,
                                self.norms, self.gnorm_sq, 0, 0.0, 1.0)
        elif self.kind == "lars":
            self.norms.zero_()
            ext.opt_lars_norms(s.master, s.grad, rows, self.hyper, self.gnorm_sq, self.norms)
            if red is not None:
                red.sum_(self.norms)
            ext.opt_apply_trust(s.master, s.grad, self.trace, shadow, rows, self.meta, self.hyper,
                                self.norms, self.gnorm_sq, 1, self.momentum, self.trust_coefficient)
        else:
            ext.opt_sgd(s.master, s.grad, self.trace, shadow, rows, self.meta, self.hyper,
                        self.gnorm_sq, self.momentum)

    # ---------------------------------------------------------------- state io
    def state_dict(self) -> dict:
        d = {"kind": self.kind, "count": self.count}
        for k in ("mu", "nu", "trace"):
            v = getattr(self, k)
            if v is not None:
                d[k] = v.detach().cpu()
        return d

    def load_state_dict(self, d: dict) -> None:
        assert d["kind"] == self.kind
        self.count = int(d["count"])
        for k in ("mu", "nu", "trace"):
            dst = getattr(self, k)
            if k not in d or dst is None:
                continue
            src = d[k].reshape(-1)
            # segment offsets do not depend on the flat total's padding (models/params.py
            # TOTAL_ALIGN; earlier builds padded to 64): copy the common prefix, zero the rest.
            # Everything past the last segment is padding, which is never read as a parameter.
            n = min(src.numel(), dst.numel())
            if src.numel() > n and bool(src[n:].any()):
                raise ValueError(f"optimizer state '{k}' has {src.numel()} elements with non-zero entries "
                                 f"past this store's {dst.numel()}")
            if n < self.store.used_numel():
                raise ValueError(f"optimizer state '{k}' has {src.numel()} elements; the parameters span "
                                 f"{self.store.used_numel()}")
            dst[:n].copy_(src[:n])
            dst[n:].zero_()
        self.last_lr = self.schedule(max(self.count - 1, 0))
