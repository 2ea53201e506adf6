"""Data-parallel gradient reducer over the flat fp32 gradient buffer, overlapped with backward.

Reference: ``jax.lax.pmean(grads, axis_name="batch")`` inside the pmap'd training step
(/root/reference/src/pretraining.py:150, finetuning.py:144).

MI355X design:
* The gradient buffer is ONE contiguous fp32 allocation whose segment order is the reverse of
  backward readiness (models build params in forward order).  Buckets are contiguous slices
  cut from the end of the buffer, so bucket k becomes complete while backward is still
  computing bucket k+1 -- no packing copies, RCCL reduces the buffer in place.
* Readiness is counted per segment: every forward use of a parameter bumps its pending count,
  every backward write decrements it (``Handle.ready``), so a weight shared by all layers --
  the jumbo MLP -- is reduced only after its last (layer-0) contribution.
* When a bucket is complete its ``all_reduce(AVG)`` is issued asynchronously on RCCL's stream;
  ``finish()`` waits for all of them (and flushes buckets that had unused segments).
* Bucket size defaults to 64 MiB: large enough for the ring's bandwidth regime on xGMI
  (7 links x ~150 GB/s per MI355X), small enough that the first bucket starts early.
* With ``grad_accum > 1`` call ``set_sync(False)`` on the non-final micro-steps (no-sync
  accumulation, CC2).
* Partial readiness: the shared jumbo-MLP weights are final only at the very end of backward
  (their batched weight-gradient GEMM runs after layer 0).  Their GEMM is split into row chunks
  (ops/prims.py flush_deferred_wgrads) and each chunk's slice is all-reduced as soon as it is
  written (``ParamStore.mark_partial_ready``), so only the last chunk's reduction is exposed
  instead of two 150 MB tensors (ViT-L).  Only single-segment buckets take partial launches.
"""

from __future__ import annotations

import contextlib
import os

import torch
import torch.distributed as dist

from ..models.params import Handle, ParamStore
from . import dist as pdist


class GradReducer:
    def __init__(self, store: ParamStore, group=None, bucket_mb: float = 64.0, overlap: bool = True,
                 reduce_dtype: torch.dtype = torch.float32, seg_filter=None):
        self.store = store
        self.group = group
        self.world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
        from .dist import forced_group

        self.enabled = self.world > 1 or (forced_group() and dist.is_available() and dist.is_initialized())
        # JMAE_REDUCER_OVERLAP=0: every bucket is launched from finish() (diagnostics / A/B)
        self.overlap = overlap and self.enabled and os.environ.get("JMAE_REDUCER_OVERLAP", "1") == "1"
        self.sync = True
        self.reduce_dtype = reduce_dtype
        segs = [s for s in store.segments if s.trainable and (seg_filter is None or seg_filter(s))]
        self.seg_index = {id(s): i for i, s in enumerate(segs)}
        # -------- buckets from the end of the flat buffer
        limit = int(bucket_mb * 1024 * 1024 / 4)
        buckets: list[list[int]] = []
        cur: list[int] = []
        size = 0
        for i in range(len(segs) - 1, -1, -1):
            s = segs[i]
            if cur and size + s.numel > limit:
                buckets.append(cur)
                cur, size = [], 0
            cur.append(i)
            size += s.numel
        if cur:
            buckets.append(cur)
        self.segs = segs
        self.buckets = []
        self.seg_bucket = [0] * len(segs)
        for bi, idxs in enumerate(buckets):
            lo = min(segs[i].offset for i in idxs)
            hi = max(segs[i].offset + segs[i].numel for i in idxs)
            self.buckets.append((lo, hi, idxs))
            for i in idxs:
                self.seg_bucket[i] = bi
        self.pending_uses = [0] * len(segs)
        self.bucket_left = [len(b[2]) for b in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.works = []
        self._compressed = {}
        self.partial_done = [0] * len(self.buckets)  # elements of a bucket already launched
        if self.enabled:
            store.hooks.append(self._on_ready)
            store.use_hooks.append(self._on_use)
            store.partial_hooks.append(self._on_partial)

    # ---------------------------------------------------------------- protocol
    def set_sync(self, sync: bool) -> None:
        self.sync = sync

    def begin_step(self) -> None:
        self.pending_uses = [0] * len(self.segs)
        self.bucket_left = [len(b[2]) for b in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.partial_done = [0] * len(self.buckets)
        self.works = []

    def _on_partial(self, h: Handle, lo: int, hi: int) -> None:
        """Elements [lo, hi) of single-segment handle ``h`` are final: reduce them now."""
        if not (self.overlap and self.sync) or len(h.segs) != 1:
            return
        i = self.seg_index.get(id(h.segs[0]))
        if i is None:
            return
        b = self.seg_bucket[i]
        blo, bhi, idxs = self.buckets[b]
        if len(idxs) != 1 or self.launched[b] or self.reduce_dtype != torch.float32:
            return
        off = self.segs[i].offset
        self.works.append((b, self._allreduce(self.store.grad[off + lo:off + hi])))
        self.partial_done[b] += hi - lo

    def _on_use(self, h: Handle) -> None:
        # only the synchronising micro-step's uses are matched by counted backward writes
        # (``_on_ready`` ignores no-sync micro-steps); counting the others would keep
        # ``pending_uses`` above 0 and push every bucket to ``finish()`` (no overlap)
        if not self.sync:
            return
        for s in h.segs:
            i = self.seg_index.get(id(s))
            if i is not None:
                self.pending_uses[i] += 1

    def _on_ready(self, h: Handle) -> None:
        if not (self.overlap and self.sync):
            return
        for s in h.segs:
            i = self.seg_index.get(id(s))
            if i is None:
                continue
            self.pending_uses[i] -= 1
            if self.pending_uses[i] == 0:
                b = self.seg_bucket[i]
                self.bucket_left[b] -= 1
                if self.bucket_left[b] == 0:
                    self._launch(b)

    def _launch(self, b: int) -> None:
        if self.launched[b]:
            return
        self.launched[b] = True
        lo, hi, _ = self.buckets[b]
        if self.partial_done[b]:
            if self.partial_done[b] != hi - lo:
                raise RuntimeError(f"bucket {b}: partial reductions cover {self.partial_done[b]} of {hi - lo}")
            return
        view = self.store.grad[lo:hi]
        if self.reduce_dtype != torch.float32:
            buf = view.to(self.reduce_dtype)
            self._compressed[b] = buf
            w = self._allreduce(buf)
        else:
            w = self._allreduce(view)
        self.works.append((b, w))

    def _allreduce(self, t: torch.Tensor):
        """Async all-reduce-average of ``t`` -> (work, tensor to divide by world or None).  One code
        path for every backend: only the reduction op differs (RCCL averages inside the
        collective, gloo has no AVG and is divided after the wait).  On a GPU the collective is
        issued from the weight-gradient stream (ops/prims.py) when that stream is enabled, after
        it has caught up with the main stream: RCCL then waits for the GEMM that wrote the
        bucket's last kernel gradient without stalling the backward chain on the main stream."""
        from ..ops.prims import wgrad_stream
        native_avg = dist.get_backend(self.group) == "nccl"
        op = dist.ReduceOp.AVG if native_avg else dist.ReduceOp.SUM
        side = wgrad_stream() if t.is_cuda else None
        if side is not None:
            side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            w = dist.all_reduce(t, op=op, group=self.group, async_op=True)
        return w, (None if native_avg else t)

    def bucket_ranges(self) -> list[tuple[int, int]]:
        return [(lo, hi) for lo, hi, _ in self.buckets]

    def optimizer_groups(self) -> list[list[int]]:
        """Consecutive bucket indices whose optimizer update is issued as ONE launch once all of
        them are reduced (``JMAE_OPT_GROUPS``, default 4; 0 = one launch per bucket).  Buckets are
        contiguous flat ranges in launch order, so a group is one contiguous range.  Measured at one
        rank on RCCL: 30 per-bucket AdamW launches cost 0.4 ms/step more than one
        (profiles/r2_dp_overhead_1rank.txt); a few groups keep the update of the early buckets
        overlapped with the reduction of the last ones."""
        nb = len(self.buckets)
        g = int(os.environ.get("JMAE_OPT_GROUPS", "4"))
        g = nb if g <= 0 else max(1, min(g, nb))
        return [list(range(nb * i // g, nb * (i + 1) // g)) for i in range(g)]

    def optimizer_ranges(self) -> list[tuple[int, int]]:
        return [(min(self.buckets[b][0] for b in grp), max(self.buckets[b][1] for b in grp))
                for grp in self.optimizer_groups()]

    def finish(self, on_bucket_done=None) -> None:
        """Launch any bucket not yet reduced (unused segments / no overlap) and wait for all.

        ``on_bucket_done(lo, hi)`` is called as soon as the last reduction of an optimizer group
        (``optimizer_ranges``, consecutive buckets) has been
        waited for (on RCCL: a stream wait, the host does not block), so the caller can queue
        the optimizer update of that range behind it while later buckets -- the jumbo-MLP tail
        -- are still being reduced."""
        from ..ops.prims import join_wgrad_stream
        join_wgrad_stream()
        if not self.enabled or not self.sync:
            return
        for b in range(len(self.buckets)):
            if not self.launched[b]:
                self._launch(b)
        groups = self.optimizer_groups()
        ranges = self.optimizer_ranges()
        gid = {b: i for i, grp in enumerate(groups) for b in grp}
        left = [0] * len(groups)  # outstanding reductions per optimizer group
        for b, _ in self.works:
            left[gid[b]] += 1
        for b, (w, to_div) in self.works:
            w.wait()
            if to_div is not None:
                to_div.div_(self.world)
            if b in self._compressed:
                lo, hi, _ = self.buckets[b]
                self.store.grad[lo:hi].copy_(self._compressed.pop(b))
            left[gid[b]] -= 1
            if on_bucket_done is not None and left[gid[b]] == 0:
                on_bucket_done(*ranges[gid[b]])
        if on_bucket_done is not None:  # a group without any reduction of its own (none today)
            for i, grp in enumerate(groups):
                if not any(gid[b] == i for b, _ in self.works):
                    on_bucket_done(*ranges[i])
        self.works = []

    def stats(self) -> dict:
        sizes = [(hi - lo) * 4 / 2**20 for lo, hi, _ in self.buckets]
        return {"buckets": len(self.buckets), "bucket_mb_max": max(sizes) if sizes else 0.0,
                "bucket_mb_min": min(sizes) if sizes else 0.0}
