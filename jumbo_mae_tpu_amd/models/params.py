"""Flat parameter store: fp32 master / compute-dtype shadow / fp32 gradient in three flat buffers.

Design (MI355X-first, no reference counterpart): every Flax leaf of the reference parameter
tree is one *segment* of three contiguous device buffers:

* ``master``  fp32, what the optimizer updates (the reference keeps fp32 params),
* ``shadow``  bf16 copy read by the GEMM / attention kernels; it is rewritten by the fused
  optimizer kernel in the same pass that updates the master, so no per-step cast kernel is
  needed (a weight shared by all layers -- the jumbo MLP -- is therefore cast zero times),
* ``grad``    fp32, written *directly* by the backward kernels (wgrad GEMMs accumulate with
  beta=1 into it), which makes gradient accumulation across micro-steps and across the L
  uses of the shared jumbo MLP free, and lets the data-parallel reducer all-reduce contiguous
  buckets without packing copies.

Segments keep the per-leaf granularity of the Flax tree so that optimizer semantics that are
per leaf (LAMB / LARS trust ratios, the ``kernel`` weight-decay mask, layer-wise LR decay
labels) are exactly those of optax on the reference tree.  Storage layout is chosen for the
kernels (e.g. Dense kernels are stored out x in), and converted to the Flax layout only at
checkpoint time.  Segments are padded to 64 elements (256 B) so vector kernels never straddle.
"""

from __future__ import annotations

import contextlib

import math
from dataclasses import dataclass
from typing import Callable, Iterable

import numpy as np
import torch

ALIGN = 64
# the flat total is padded to a multiple of this, so every data-parallel world size that divides
# 1680 (1-8, 10, 12, 14, 15, 16, 20, 24, ...) can cut it into equal ALIGN-aligned shards
# (ZeRO-1 optimizer sharding, parallel/ddp.py); costs at most 420 KB per fp32 buffer.  Other
# world sizes are folded in at finalize() when the process group exists.
TOTAL_ALIGN = ALIGN * 1680


@dataclass
class Segment:
    path: tuple[str, ...]
    shape: tuple[int, ...]  # storage shape
    flax_shape: tuple[int, ...]
    to_flax: Callable[[np.ndarray], np.ndarray]
    from_flax: Callable[[np.ndarray], np.ndarray]
    init: Callable[[torch.Generator, tuple[int, ...]], torch.Tensor]
    offset: int = 0
    trainable: bool = True
    use_count: int = 0  # backward uses per step, for the reducer readiness protocol

    @property
    def numel(self) -> int:
        return int(math.prod(self.shape))

    @property
    def key(self) -> str:
        return "/".join(self.path)

    @property
    def is_kernel(self) -> bool:
        """optax mask used by the reference: leaf key == "kernel" (pretraining.py:230)."""
        return self.path[-1] == "kernel"


def identity(a: np.ndarray) -> np.ndarray:
    return a


# store-mode gradients (ParamStore.zero_grad; False zeroes the whole buffer: A/B and tests)
STORE_GRADS = True

# Handle.weight_t copies refreshed in one batched launch (False: one launch per copy)
BATCH_TRANSPOSES = True


class Handle:
    """A view over one or more *adjacent* segments (e.g. wq|wk|wv as one QKV weight)."""

    def __init__(self, store: "ParamStore", segs: list[Segment], shape: tuple[int, ...]):
        self.store = store
        self.segs = segs
        self.shape = shape
        self.start = segs[0].offset
        self.numel = int(math.prod(shape))
        for a, b in zip(segs[:-1], segs[1:]):
            assert b.offset == a.offset + a.numel, "fused handle segments must be contiguous"
        assert self.numel == sum(s.numel for s in segs)
        self._param: torch.nn.Parameter | None = None
        self._wt: torch.Tensor | None = None
        self._wt_version = -1
        self.defer_wgrad = False   # batch this weight's gradient GEMMs (weights shared by layers)
        self.deferred: list = []   # queued (dy, x) pairs of the current backward pass
        # store-mode gradient (ParamStore.zero_grad): registered once its weight gradient ran on the
        # store-capable TN path; _fresh = its grad was not zeroed this step and not written yet
        self._store_reg = False
        self._fresh = False

    def _view(self, flat: torch.Tensor) -> torch.Tensor:
        return flat[self.start:self.start + self.numel].view(self.shape)

    @property
    def master(self) -> torch.Tensor:
        return self._view(self.store.master)

    @property
    def shadow(self) -> torch.Tensor:
        return self._view(self.store.shadow)

    @property
    def grad(self) -> torch.Tensor:
        return self._view(self.store.grad)

    @property
    def param(self) -> torch.nn.Parameter:
        """Leaf tensor aliasing the master storage; passed to autograd Functions as an input
        so autograd records the op (its gradient is never returned through autograd)."""
        if self._param is None or self._param.data_ptr() != self.master.data_ptr():
            self._param = torch.nn.Parameter(self.master, requires_grad=self.segs[0].trainable)
        return self._param

    def weight(self) -> torch.Tensor:
        """Tensor the compute kernels read (bf16 shadow on GPU, master on fp32 runs)."""
        return self.shadow

    def weight_t(self) -> torch.Tensor:
        """Transposed copy of ``weight()`` ([in, out] for a Dense kernel stored out x in), the
        K-contiguous B operand of a data-gradient GEMM on the NT MFMA kernel.  Refreshed lazily
        once per shadow update (``ParamStore.version``)."""
        if self._wt is None or self._wt_version != self.store.version:
            w = self.weight()
            first = self._wt is None
            if first:
                self._wt = torch.empty((w.shape[1], w.shape[0]), dtype=w.dtype, device=w.device)
            from ..ops import _ext  # noqa: PLC0415 (models must import without the extension)
            hip_ok = _ext.use_hip(w) and w.dtype == torch.bfloat16 and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0
            if hip_ok and not first and self.store.refresh_transposes():
                return self._wt  # refreshed together with every other stale transposed copy
            if hip_ok:
                _ext.load().transpose_bf16(w, self._wt)
            else:
                self._wt.copy_(w.t())
            self._wt_version = self.store.version
        return self._wt

    def accumulate_grad(self, g: torch.Tensor) -> None:
        if not self.segs[0].trainable:
            return
        self.settle()  # a store-registered gradient skipped by zero_grad holds last step's values
        self.grad.add_(g.reshape(self.shape).to(torch.float32))
        self.store.mark_ready(self)

    def accumulate_grad_rows(self, x: torch.Tensor) -> None:
        """grad += x.sum(0) for a 2-D fp32 [rows, numel] view (any row stride): on the GPU one HIP
        column-sum kernel adding straight into the flat gradient -- no torch reduce (whose
        cross-block accumulator is zeroed by a runtime memset, a graph node that replays wrong on
        ROCm 7.x, profiles/r4_graph_memset.txt) and no separate add."""
        if not self.segs[0].trainable:
            return
        self.settle()
        from ..ops import _ext
        if (_ext.use_hip(x) and x.dtype == torch.float32 and x.stride(-1) == 1 and x.shape[-1] % 4 == 0
                and x.stride(0) % 4 == 0 and x.data_ptr() % 16 == 0):
            _ext.load().colsum_add_f32(x, self.grad.view(-1))
        else:
            self.grad.add_(x.sum(0).reshape(self.shape).to(torch.float32))
        self.store.mark_ready(self)

    def ready(self) -> None:
        self.store.mark_ready(self)

    def take_store(self) -> bool:
        """Called by a weight-gradient kernel that can overwrite this gradient: True = store (the
        first contribution since zero_grad skipped it), False = accumulate.  Registers the handle,
        so the next zero_grad leaves its range to the store."""
        if not self._store_reg:
            self.store.register_store(self)
            return False
        fresh, self._fresh = self._fresh, False
        return fresh

    def settle(self) -> None:
        """Before an accumulating write by a path that cannot store: zero a skipped gradient."""
        if self._fresh:
            self.grad.zero_()
            self._fresh = False

    def note_use(self) -> None:
        """Record one differentiable forward use (the reducer expects one ``ready`` per use)."""
        if self.store.use_hooks and self.store.count_uses and self.segs[0].trainable and torch.is_grad_enabled():
            for fn in self.store.use_hooks:
                fn(self)


class ParamStore:
    def __init__(self):
        self.segments: list[Segment] = []
        self.by_key: dict[str, Segment] = {}
        self.master: torch.Tensor | None = None
        self.shadow: torch.Tensor | None = None
        self.grad: torch.Tensor | None = None
        self.total = 0
        self.finalized = False
        self.compute_dtype = torch.float32
        self.hooks: list[Callable[[Handle], None]] = []
        self.use_hooks: list[Callable[[Handle], None]] = []
        # partial readiness: fn(handle, lo, hi) -- elements [lo, hi) of a single-segment handle's
        # gradient are final (the DP reducer may start reducing that slice early)
        self.partial_hooks: list[Callable[[Handle, int, int], None]] = []
        self._handles: list[Handle] = []
        self.count_uses = True  # off while an activation-checkpoint recompute re-runs a forward
        # store-mode gradients (zero_grad skips the TN-kernel gradients, their first write stores);
        # runtime/graph.py turns it off for captured steps
        self.allow_store = True
        self.version = 0  # bumped whenever the shadow changes (optimizer step, sync, load)
        # batched refresh of the transposed weight copies (Handle.weight_t): device descriptor
        # table, cached per set of copies
        self._wt_batch: tuple | None = None
        self._store_handles: list[Handle] = []  # zero_grad leaves these to their first (storing) write
        self._zero_plan: tuple | None = None
        self._retired_plans: list[tuple] = []  # superseded plans stay alive (a graph may read them)

    def refresh_transposes(self) -> bool:
        """Rewrite every existing transposed weight copy from the current bf16 shadow in ONE
        launch (the first ``weight_t`` call after a shadow update triggers it; the backward then
        finds all copies fresh).  Returns False when batching is off / not applicable."""
        if not BATCH_TRANSPOSES:
            return False
        # the batch kernel's 16-byte vector accesses need the single-transpose kernel's preconditions
        hs = [h for h in self._handles if h._wt is not None and h._wt.dtype == torch.bfloat16 and h._wt.is_cuda
              and len(h.shape) == 2 and h.shape[0] % 8 == 0 and h.shape[1] % 8 == 0]
        if not hs:
            return False
        key = tuple((h._wt.data_ptr(), h.shadow.data_ptr()) for h in hs)
        if self._wt_batch is None or self._wt_batch[0] != key:
            rows, tiles = [], 0
            for h in hs:
                R, C = h.shape
                ntc = -(-C // 64)
                rows.append([h.shadow.data_ptr(), h._wt.data_ptr(), R, C, tiles, ntc])
                tiles += ntc * -(-R // 64)
            desc = torch.tensor(rows, dtype=torch.int64).to(hs[0]._wt.device)
            self._wt_batch = (key, desc, tiles)
        from ..ops import _ext  # noqa: PLC0415
        _ext.load().transpose_bf16_batch(self._wt_batch[1], self._wt_batch[2])
        for h in hs:
            h._wt_version = self.version
        return True

    @contextlib.contextmanager
    def uses_suppressed(self):
        """Forward re-runs (activation-checkpoint recompute) record no parameter uses."""
        prev, self.count_uses = self.count_uses, False
        try:
            yield
        finally:
            self.count_uses = prev

    # ---------------------------------------------------------------- building
    def add(self, path: Iterable[str], shape: tuple[int, ...], init, flax_shape=None,
            to_flax=identity, from_flax=identity, trainable: bool = True) -> Segment:
        assert not self.finalized
        path = tuple(path)
        seg = Segment(path=path, shape=tuple(shape), flax_shape=tuple(flax_shape or shape),
                      to_flax=to_flax, from_flax=from_flax, init=init, trainable=trainable)
        key = seg.key
        assert key not in self.by_key, f"duplicate param {key}"
        seg.offset = self.total
        self.total += seg.numel
        self.segments.append(seg)
        self.by_key[key] = seg
        return seg

    def pad(self) -> None:
        """Align the next segment to ALIGN elements (keeps fused handles contiguous otherwise)."""
        self.total = (self.total + ALIGN - 1) // ALIGN * ALIGN

    def handle(self, segs: list[Segment] | Segment, shape: tuple[int, ...] | None = None) -> Handle:
        if isinstance(segs, Segment):
            segs = [segs]
        h = Handle(self, segs, tuple(shape) if shape is not None else segs[0].shape)
        self._handles.append(h)
        return h

    def used_numel(self) -> int:
        """Elements up to the end of the last segment (the flat total adds alignment padding)."""
        return max((s.offset + s.numel for s in self.segments), default=0)

    def finalize(self, device, compute_dtype=torch.float32, generator: torch.Generator | None = None) -> None:
        q = TOTAL_ALIGN
        # a data-parallel world that does not divide 1680 (32, 64 ranks) still gets equal 64-aligned
        # ZeRO-1 shards: pad to lcm(TOTAL_ALIGN, world * ALIGN)
        import torch.distributed as dist  # noqa: PLC0415
        if dist.is_available() and dist.is_initialized():
            q = math.lcm(q, dist.get_world_size() * ALIGN)
        self.total = (self.total + q - 1) // q * q
        self.compute_dtype = compute_dtype
        self.master = torch.zeros(self.total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=device)
        if compute_dtype == torch.float32:
            self.shadow = self.master
        else:
            self.shadow = torch.zeros(self.total, dtype=compute_dtype, device=device)
        self.finalized = True
        self.initialize(generator)

    def initialize(self, generator: torch.Generator | None = None) -> None:
        g = generator or torch.Generator().manual_seed(0)
        with torch.no_grad():
            for s in self.segments:
                v = s.init(g, s.shape).to(torch.float32)
                self.master[s.offset:s.offset + s.numel].copy_(v.reshape(-1))
        self.sync_shadow()

    def sync_shadow(self) -> None:
        self.version += 1
        if self.shadow is not self.master:
            with torch.no_grad():
                self.shadow.copy_(self.master)

    # ---------------------------------------------------------------- grads
    def zero_grad(self) -> None:
        """Reset the gradients for a new step.  The Dense kernels whose weight gradient runs on the
        TN MFMA kernel (registered by Handle.take_store) are NOT zeroed: their first contribution
        stores instead of adding -- the split-K reduce then skips reading the gradient too -- and
        everything else (biases, LayerNorm, embeddings: ~2 % of the bytes) is zeroed by one
        multi-range launch.  A registered gradient nobody wrote is zeroed by flush_fresh."""
        hs = self._store_handles
        if not (STORE_GRADS and self.allow_store and hs and self.grad.is_cuda):
            self.grad.zero_()
            for h in hs:
                h._fresh = False
            return
        key = tuple(h.start for h in hs)
        if self._zero_plan is None or self._zero_plan[0] != key:
            # the plan's descriptor is an H2D copy: never built inside a HIP-graph capture (a
            # captured step reuses the plan of its warmup steps; a changed handle set after
            # capture would free the descriptor the graph reads -- runtime/graph.py pins it)
            assert not torch.cuda.is_current_stream_capturing(), "zero_grad plan changed during capture"
            if self._zero_plan is not None:
                self._retired_plans.append(self._zero_plan)
            spans = sorted((h.start, h.start + h.numel) for h in hs)
            ranges, pos = [], 0
            for a, b in spans:
                if a > pos:
                    ranges.append((pos, a - pos))
                pos = max(pos, b)
            if pos < self.grad.numel():
                ranges.append((pos, self.grad.numel() - pos))
            blocks = sum(-(-c // 4096) for _, c in ranges)
            desc = torch.tensor(ranges if ranges else [(0, 0)], dtype=torch.int64).to(self.grad.device)
            self._zero_plan = (key, desc, blocks)
        from ..ops import _ext  # noqa: PLC0415
        _ext.load().zero_ranges(self.grad, self._zero_plan[1], self._zero_plan[2])
        for h in hs:
            h._fresh = True

    def register_store(self, h: Handle) -> None:
        if STORE_GRADS and self.allow_store and not h._store_reg and self.grad is not None and self.grad.is_cuda:
            h._store_reg = True
            self._store_handles.append(h)

    def flush_fresh(self) -> None:
        """After the backward: zero any skipped gradient that received no contribution."""
        for h in self._store_handles:
            h.settle()

    def mark_ready(self, h: Handle) -> None:
        for fn in self.hooks:
            fn(h)

    def mark_partial_ready(self, h: Handle, lo: int, hi: int) -> None:
        for fn in self.partial_hooks:
            fn(h, lo, hi)

    def seg_view(self, flat: torch.Tensor, seg: Segment) -> torch.Tensor:
        return flat[seg.offset:seg.offset + seg.numel].view(seg.shape)

    # ---------------------------------------------------------------- flax tree IO
    def to_flax_tree(self, prefix: tuple[str, ...] = ()) -> dict:
        tree: dict = {}
        master = self.master.detach().float().cpu().numpy()
        for s in self.segments:
            arr = master[s.offset:s.offset + s.numel].reshape(s.shape)
            arr = np.ascontiguousarray(s.to_flax(arr).astype(np.float32))
            assert tuple(arr.shape) == s.flax_shape, (s.key, arr.shape, s.flax_shape)
            node = tree
            for k in s.path[:-1]:
                node = node.setdefault(k, {})
            node[s.path[-1]] = arr
        return tree

    def load_flax_tree(self, tree: dict, strict: bool = False, subtree: tuple[str, ...] = ()) -> tuple[int, int]:
        """Copy leaves that exist in ``tree`` (and match shape). Returns (loaded, total)."""
        loaded = 0
        total = 0
        with torch.no_grad():
            for s in self.segments:
                if subtree and s.path[:len(subtree)] != subtree:
                    continue
                total += 1
                node = tree
                ok = True
                for k in s.path:
                    if isinstance(node, dict) and k in node:
                        node = node[k]
                    else:
                        ok = False
                        break
                if not ok:
                    if strict:
                        raise KeyError(s.key)
                    continue
                arr = np.asarray(node, dtype=np.float32)
                if tuple(arr.shape) != s.flax_shape:
                    if strict:
                        raise ValueError(f"shape mismatch {s.key}: {arr.shape} vs {s.flax_shape}")
                    continue
                v = torch.from_numpy(np.ascontiguousarray(s.from_flax(arr)).reshape(-1))
                self.master[s.offset:s.offset + s.numel].copy_(v)
                loaded += 1
        self.sync_shadow()
        return loaded, total

    def num_params(self, trainable_only: bool = False) -> int:
        return sum(s.numel for s in self.segments if (s.trainable or not trainable_only))


# ---------------------------------------------------------------------- initializers
def trunc_normal_(generator: torch.Generator, shape, std: float = 0.02) -> torch.Tensor:
    """jax.nn.initializers.truncated_normal(0.02): samples N(0,1) truncated to [-2,2], scaled by
    std / 0.87962566 (the std of the unit truncated normal) so the result has std ``std``."""
    # inverse-CDF sampling of the truncated normal on the generator's device (deterministic per
    # seed and device type; ranks are made identical by a broadcast from rank 0)
    lo, hi = -2.0, 2.0
    u = torch.rand(tuple(shape), generator=generator, dtype=torch.float64, device=generator.device)
    a = torch.special.ndtr(torch.tensor(lo, dtype=torch.float64, device=u.device))
    b = torch.special.ndtr(torch.tensor(hi, dtype=torch.float64, device=u.device))
    x = torch.special.ndtri(a + u * (b - a))
    x = x.clamp(lo, hi)
    return (x * (std / 0.87962566103423978)).to(torch.float32)


def zeros_(generator, shape) -> torch.Tensor:
    return torch.zeros(tuple(shape), dtype=torch.float32)


def ones_(generator, shape) -> torch.Tensor:
    return torch.ones(tuple(shape), dtype=torch.float32)


def const_(value: float):
    def f(generator, shape):
        return torch.full(tuple(shape), value, dtype=torch.float32)
    return f


def trunc_normal_t(std: float = 0.02):
    """Initializer for an out x in stored Dense kernel: draw in Flax (in, out) order, then
    transpose, so a given seed produces the same weights as a Flax-layout draw would."""
    def f(generator, shape):
        out, inn = shape[0], int(np.prod(shape[1:]))
        return trunc_normal_(generator, (inn, out), std).t().contiguous().reshape(shape)
    return f
