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
* Buckets are cut on layer boundaries (SURVEY.md §5.8 bucket plan): consecutive segments of one
  encoder / decoder layer (or of the jumbo MLP, or of one top-level module) form a unit that is
  never split across buckets unless the unit alone exceeds the bucket size; a segment larger
  than the bucket size (the jumbo MLP kernels) is a bucket of its own, so it keeps its partial
  launches.  At the 64 MiB default that is one ViT-L encoder layer (50 MB) per bucket, five
  decoder layers, and one bucket per jumbo kernel.
* ``reduce_dtype=bf16`` converts each bucket (or partial slice) into ONE preallocated bf16
  staging buffer laid out like the flat gradient buffer -- no per-step allocation -- and copies
  the averaged slice back after the collective; partial launches work the same way.
* ``shard=True`` (ZeRO-1 optimizer sharding): bucket boundaries are snapped to multiples of
  world x 64 elements (a segment cut by a boundary belongs to both buckets and both wait for it),
  so every bucket splits into ``world`` equal 64-aligned pieces and rank r owns piece r of every
  bucket.  A complete bucket is REDUCE-SCATTERED (in place: rank r's piece of the flat gradient
  receives the average), the optimizer updates only the owned pieces (1/world of the AdamW /
  LAMB / LARS / SGD work; LAMB / LARS per-leaf norms and the global clip norm are summed over the
  ranks by a tiny all-reduce), and each bucket's updated bf16 SHADOW (the compute copy the
  optimizer kernel writes beside the owned fp32 master) is ALL-GATHERED in place: 2 bytes per
  parameter on the link instead of the fp32 master's 4, no re-cast pass, bit-identical weights
  (every rank's shadow piece is the cast of its owner's new master).  The fp32 master of a
  non-owned piece is then stale on this rank -- only the owner updates it, as in ZeRO-1 -- and
  ``gather_state`` all-gathers it (with the optimizer moments) for a checkpoint / export.  The few
  parameters the kernels read in fp32 from the master (biases, LayerNorm / LayerScale, tokens:
  every non-``kernel`` leaf, ~0.1 % of a ViT) are exchanged exactly each step by one small int32
  all-reduce of their bits (``exchange_fp32``).
  ``gather_dtype="fp32"`` gathers the master and re-casts (the round-5 path; also used whenever the
  shadow IS the master, i.e. fp32 compute).  Link bytes per parameter: 4 + 2 (fp32 reduce-scatter
  + bf16 gather), 2 + 2 with ``reduce_dtype=bf16``.
* Chunked jumbo tail in ZeRO-1 mode: a reduce-scatter cannot start on a partial range of its bucket
  (rank r owns piece r of the WHOLE bucket), so a bucket holding a segment larger than the bucket
  size is cut into ``PARTIAL_SUB`` sub-buckets at the row-chunk boundaries of the batched jumbo
  weight-gradient GEMM (quarters of the segment, snapped to world x 64), each with its own
  owned pieces.  Readiness is tracked as covered element ranges per segment (whole segments from
  the use counts, row chunks from ``mark_partial_ready``); a sub-bucket is reduce-scattered as soon
  as every element of it is final, so only the last quarter's reduce-scatter waits for the end of
  the backward -- the same exposure as the all-reduce mode's partial launches.
"""

from __future__ import annotations

import contextlib
import re
import time

import torch
import torch.distributed as dist

from ..models.params import ALIGN, Handle, ParamStore


_LAYER = re.compile(r"(dec_)?layer_\d+")

# optimizer launches per step on the split (per-bucket-group) path (profiles/r2_dp_overhead_1rank.txt)
OPT_GROUPS = 4
# sub-buckets of an oversized single segment in ZeRO-1 mode: the row chunks of the batched jumbo
# weight-gradient GEMM (ops/prims.py _deferred["chunks"])
PARTIAL_SUB = 4


def split_oversized(buckets: list[tuple[int, int]], big: list[tuple[int, int]], q: int,
                    parts: int = PARTIAL_SUB) -> list[tuple[int, int]]:
    """Cut every bucket [lo, hi) that overlaps an oversized segment [off, off + n) of ``big`` at
    that segment's ``parts`` equal-size boundaries snapped down to ``q`` -> ranges, same order."""
    out = []
    for lo, hi in buckets:
        cuts = {lo, hi}
        for off, n in big:
            if off < hi and off + n > lo:
                for j in range(1, parts):
                    c = (off + n * j // parts) // q * q
                    if lo < c < hi:
                        cuts.add(c)
        cs = sorted(cuts)
        out.extend(list(zip(cs[:-1], cs[1:]))[::-1])  # launch order: from the end of the buffer
    return out


def _cover(ivs: list[tuple[int, int]], lo: int, hi: int) -> bool:
    """[lo, hi) inside the union of the (merged, sorted) intervals ``ivs``."""
    for a, b in ivs:
        if a <= lo < b:
            return hi <= b
    return lo >= hi


def _merge(ivs: list[tuple[int, int]], a: int, b: int) -> list[tuple[int, int]]:
    out = []
    for x, y in sorted(ivs + [(a, b)]):
        if out and x <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], y))
        else:
            out.append((x, y))
    return out


def unit_key(path: tuple[str, ...]) -> tuple[str, ...]:
    """Bucketing unit of a parameter: its encoder / decoder layer, the shared jumbo MLP, or (for
    everything else) its top-level module."""
    for i, p in enumerate(path):
        if p == "jumbo_mlp" or _LAYER.fullmatch(p):
            return tuple(path[:i + 1])
    return tuple(path[:2])


def plan_buckets(sizes: list[int], keys: list[tuple], limit: int) -> list[list[int]]:
    """Buckets (lists of segment indices, in launch order = from the END of the buffer) of at most
    ``limit`` elements where possible: consecutive segments with one key form a unit that goes
    into one bucket; a unit larger than ``limit`` is split greedily, and a segment larger than
    ``limit`` is a bucket of its own."""
    units: list[list[int]] = []
    for i, k in enumerate(keys):
        if units and keys[units[-1][0]] == k:
            units[-1].append(i)
        else:
            units.append([i])
    buckets: list[list[int]] = []
    cur: list[int] = []
    size = 0

    def flush():
        nonlocal cur, size
        if cur:
            buckets.append(cur)
        cur, size = [], 0

    for u in reversed(units):
        usize = sum(sizes[i] for i in u)
        if usize <= limit:
            if cur and size + usize > limit:
                flush()
            cur.extend(reversed(u))
            size += usize
            continue
        flush()
        for i in reversed(u):
            if sizes[i] > limit:
                flush()
                buckets.append([i])
                continue
            if cur and size + sizes[i] > limit:
                flush()
            cur.append(i)
            size += sizes[i]
        flush()
    flush()
    return buckets


def shard_ranges(buckets: list[tuple[int, int]], q: int) -> list[tuple[int, int]]:
    """Bucket ranges with every boundary snapped DOWN to a multiple of ``q`` (the first start too,
    the last end UP), in launch order (from the end of the buffer).  The ranges tile
    [first start, last end); a bucket whose snapped boundary does not advance merges into the next."""
    asc = sorted(buckets)
    cuts = [asc[0][0] // q * q]
    for _, hi in asc[:-1]:
        c = hi // q * q
        if c > cuts[-1]:
            cuts.append(c)
    end = -(-asc[-1][1] // q) * q
    if end > cuts[-1]:
        cuts.append(end)
    return list(zip(cuts[:-1], cuts[1:]))[::-1]


class GradReducer:
    def __init__(self, store: ParamStore, group=None, bucket_mb: float = 64.0, overlap: bool = True,
                 reduce_dtype: torch.dtype = torch.float32, seg_filter=None, shard: bool = False,
                 gather_dtype: str = "bf16"):
        self.store = store
        self.group = group
        self.world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
        from .dist import forced_group

        self.enabled = self.world > 1 or (forced_group() and dist.is_available() and dist.is_initialized())
        self.overlap = overlap and self.enabled
        self.sync = True
        self.reduce_dtype = reduce_dtype
        segs = [s for s in store.segments if s.trainable and (seg_filter is None or seg_filter(s))]
        self.seg_index = {id(s): i for i, s in enumerate(segs)}
        # -------- buckets from the end of the flat buffer, cut on unit (layer) boundaries
        limit = max(int(bucket_mb * 1024 * 1024 / 4), 1)
        buckets = plan_buckets([s.numel for s in segs], [unit_key(s.path) for s in segs], limit)
        self.segs = segs
        self.buckets = []
        for idxs in buckets:
            lo = min(segs[i].offset for i in idxs)
            hi = max(segs[i].offset + segs[i].numel for i in idxs)
            self.buckets.append((lo, hi, idxs))
        self.shard = bool(shard) and self.enabled and bool(self.buckets)
        self.rank = dist.get_rank(group) if self.enabled else 0
        if self.shard:
            q = self.world * ALIGN
            if store.total % q:
                raise ValueError(f"optimizer sharding over {self.world} ranks needs the flat total ({store.total}) "
                                 f"to be a multiple of {q}: build the model after init_process_group "
                                 f"(models/params.py ParamStore.finalize pads for the world size)")
            ranges = shard_ranges([(lo, hi) for lo, hi, _ in self.buckets], q)
            ranges = split_oversized(ranges, [(s.offset, s.numel) for s in segs if s.numel > limit], q)
            self.buckets = [(lo, hi, [i for i, s in enumerate(segs) if s.offset < hi and s.offset + s.numel > lo])
                            for lo, hi in ranges]
        self.seg_buckets: list[list[int]] = [[] for _ in segs]  # a snapped boundary may cut a segment
        for bi, (_, _, idxs) in enumerate(self.buckets):
            for i in idxs:
                self.seg_buckets[i].append(bi)
        # ZeRO-1 all-gathers the bf16 shadow (the master stays sharded between checkpoints)
        self.gather_shadow = self.shard and gather_dtype == "bf16" and store.shadow is not store.master
        self._fp32_idx = None
        self.gathers: list[tuple] = []  # (bucket, work) all-gathers of the updated weights (shard)
        self.gathered = [False] * len(self.buckets)
        self._stage = None  # bf16 staging buffer over [stage_lo, stage_hi) of the flat buffer
        self._stage_lo = min((lo for lo, _, _ in self.buckets), default=0)
        self._stage_hi = max((hi for _, hi, _ in self.buckets), default=0)
        if self.gather_shadow:
            self._init_fp32_exchange()
        self.pending_uses = [0] * len(segs)
        self.ready_iv: list[list[tuple[int, int]]] = [[] for _ in segs]  # shard: final element ranges
        self.bucket_left = [len(b[2]) for b in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.works: list[tuple] = []  # (bucket, work, tensor to divide or None, lo, hi, staged, partial)
        self.partial_done = [0] * len(self.buckets)  # elements of a bucket already launched
        # readiness trace (bench.py calibration step): a list -> (bucket, lo, hi, partial, event)
        # per collective launch, the event recorded on the compute stream when the range was final
        self.trace_events: list | None = None
        if self.enabled:
            store.hooks.append(self._on_ready)
            store.use_hooks.append(self._on_use)
            store.partial_hooks.append(self._on_partial)

    # ---------------------------------------------------------------- protocol
    def set_sync(self, sync: bool) -> None:
        self.sync = sync

    def begin_step(self) -> None:
        self.pending_uses = [0] * len(self.segs)
        self.ready_iv = [[] for _ in self.segs]
        self.bucket_left = [len(b[2]) for b in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.partial_done = [0] * len(self.buckets)
        self.works = []
        self.gathers = []
        self.gathered = [False] * len(self.buckets)

    def piece(self, b: int) -> tuple[int, int]:
        """This rank's piece [lo, hi) of bucket ``b`` (sharded mode; the whole bucket otherwise)."""
        lo, hi, _ = self.buckets[b]
        if not self.shard:
            return lo, hi
        n = (hi - lo) // self.world
        return lo + self.rank * n, lo + (self.rank + 1) * n

    def _shard_ready(self, i: int, lo: int, hi: int) -> None:
        """ZeRO-1: elements [lo, hi) of segment ``i`` are final; reduce-scatter every bucket of that
        segment whose elements are now all final (``split_oversized`` sub-buckets)."""
        self.ready_iv[i] = _merge(self.ready_iv[i], lo, hi)
        for b in self.seg_buckets[i]:
            if self.launched[b]:
                continue
            blo, bhi, idxs = self.buckets[b]
            if all(_cover(self.ready_iv[j], max(blo, self.segs[j].offset) - self.segs[j].offset,
                          min(bhi, self.segs[j].offset + self.segs[j].numel) - self.segs[j].offset)
                   for j in idxs):
                self._launch(b)

    def _on_partial(self, h: Handle, lo: int, hi: int) -> None:
        """Elements [lo, hi) of single-segment handle ``h`` are final: reduce them now."""
        if not (self.overlap and self.sync) or len(h.segs) != 1:
            return
        i = self.seg_index.get(id(h.segs[0]))
        if i is None:
            return
        if self.shard:
            self._shard_ready(i, lo, hi)
            return
        b = self.seg_buckets[i][0]
        blo, bhi, idxs = self.buckets[b]
        if len(idxs) != 1 or self.launched[b]:
            return
        off = self.segs[i].offset
        self._reduce_range(b, off + lo, off + hi, partial=True)
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
            if self.pending_uses[i] == 0 and self.shard:
                self._shard_ready(i, 0, s.numel)
            elif self.pending_uses[i] == 0:
                for b in self.seg_buckets[i]:
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
        self._reduce_range(b, lo, hi)

    def staging(self) -> torch.Tensor | None:
        """The bf16 staging buffer (allocated once, on the gradient buffer's device)."""
        if self.reduce_dtype == torch.float32:
            return None
        if self._stage is None:
            self._stage = torch.empty(self._stage_hi - self._stage_lo, dtype=self.reduce_dtype,
                                      device=self.store.grad.device)
        return self._stage

    def _reduce_range(self, b: int, lo: int, hi: int, partial: bool = False) -> None:
        """Launch the all-reduce of flat-buffer elements [lo, hi) (bucket ``b``); sharded: the
        in-place reduce-scatter whose result lands in this rank's piece."""
        view = self.store.grad[lo:hi]
        if self.trace_events is not None:
            ev = torch.cuda.Event(enable_timing=True) if view.is_cuda else None
            if ev is not None:
                ev.record()
            self.trace_events.append((b, lo, hi, partial, ev if ev is not None else time.perf_counter()))
        st = self.staging()
        if self.shard:
            plo, phi = self.piece(b)
            src = view
            if st is not None:
                src = st[lo - self._stage_lo:hi - self._stage_lo]
                src.copy_(view)
            out = src[plo - lo:phi - lo]
            w, to_div = self._collective(lambda op: dist.reduce_scatter_tensor(out, src, op=op, group=self.group,
                                                                                async_op=True), out)
            self.works.append((b, w, to_div, plo, phi, out if st is not None else None, False))
            return
        if st is not None:
            sv = st[lo - self._stage_lo:hi - self._stage_lo]
            sv.copy_(view)
            w, to_div = self._allreduce(sv)
            self.works.append((b, w, to_div, lo, hi, sv, partial))
        else:
            w, to_div = self._allreduce(view)
            self.works.append((b, w, to_div, lo, hi, None, partial))

    def _allreduce(self, t: torch.Tensor):
        """Async all-reduce-average of ``t`` -> (work, tensor to divide by world or None).  One code
        path for every backend: only the reduction op differs (RCCL averages inside the
        collective, gloo has no AVG and is divided after the wait).  On a GPU the collective is
        issued from the weight-gradient stream (ops/prims.py) when that stream is enabled, after
        it has caught up with the main stream: RCCL then waits for the GEMM that wrote the
        bucket's last kernel gradient without stalling the backward chain on the main stream."""
        return self._collective(lambda op: dist.all_reduce(t, op=op, group=self.group, async_op=True), t)

    def _collective(self, issue, t: torch.Tensor):
        """Issue an averaging collective (``issue(op)``) whose result is ``t``, on the
        weight-gradient stream when there is one (see _allreduce) -> (work, tensor to divide)."""
        from ..ops.prims import wgrad_stream
        native_avg = dist.get_backend(self.group) == "nccl"
        op = dist.ReduceOp.AVG if native_avg else dist.ReduceOp.SUM
        side = wgrad_stream() if t.is_cuda else None
        if side is not None:
            side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            w = issue(op)
        return w, (None if native_avg else t)

    # ---------------------------------------------------------------- sharded optimizer (ZeRO-1)
    def owned_pieces(self, buckets=None) -> list[tuple[int, int]]:
        return [self.piece(b) for b in (range(len(self.buckets)) if buckets is None else buckets)]

    def _gather_into(self, flat: torch.Tensor, b: int):
        lo, hi, _ = self.buckets[b]
        plo, phi = self.piece(b)
        out = flat[lo:hi]
        inp = flat[plo:phi]
        side = None
        if flat.is_cuda:
            from ..ops.prims import wgrad_stream
            side = wgrad_stream() or torch.cuda.current_stream()
            if side is not torch.cuda.current_stream():
                side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            return dist.all_gather_into_tensor(out, inp, group=self.group, async_op=True)

    def _init_fp32_exchange(self) -> None:
        """The parameters the kernels read in fp32 from the MASTER (biases, LayerNorm / LayerScale
        parameters, CLS / mask tokens, learnable position embeddings: every leaf that is not a Dense
        or conv ``kernel``) must be whole on every rank even when only the bf16 shadow is gathered.
        Their elements (~0.1 % of a ViT) are exchanged each step by one int32 SUM all-reduce of
        their bits, each rank contributing its owned elements and zeros: exact, bit for bit."""
        idx, own = [], []
        owned = torch.zeros(self.store.total, dtype=torch.bool)
        for b in range(len(self.buckets)):
            lo, hi = self.piece(b)
            owned[lo:hi] = True
        for sg in self.segs:
            if sg.path[-1] == "kernel" and len(sg.shape) >= 2:
                continue
            r = torch.arange(sg.offset, sg.offset + sg.numel)
            idx.append(r)
            own.append(owned[r])
        if not idx:
            return
        dev = self.store.master.device
        self._fp32_idx = torch.cat(idx).to(dev)
        self._fp32_own = torch.cat(own).to(dev)

    def exchange_fp32(self) -> None:
        """COLLECTIVE: the owners' updated fp32 values of the master-read parameters to every rank."""
        if self._fp32_idx is None:
            return
        m = self.store.master
        bits = m[self._fp32_idx].view(torch.int32)
        bits = torch.where(self._fp32_own, bits, torch.zeros_like(bits))
        dist.all_reduce(bits, op=dist.ReduceOp.SUM, group=self.group)
        m[self._fp32_idx] = bits.view(torch.float32)

    def gather(self, b: int) -> None:
        """All-gather bucket ``b``'s updated weights (in place) after the owned piece's update: the
        bf16 shadow (``gather_shadow``) or the fp32 master."""
        if not self.shard or self.gathered[b]:
            return
        self.gathered[b] = True
        flat = self.store.shadow if self.gather_shadow else self.store.master
        self.gathers.append((b, self._gather_into(flat, b)))

    def gather_all(self) -> None:
        for b in range(len(self.buckets)):
            self.gather(b)

    def wait_gathers(self) -> None:
        """Wait for the master all-gathers and re-cast the gathered ranges to the bf16 shadow."""
        s = self.store
        for b, w in self.gathers:
            w.wait()
            if s.shadow is not s.master and not self.gather_shadow:
                lo, hi, _ = self.buckets[b]
                with torch.no_grad():
                    s.shadow[lo:hi].copy_(s.master[lo:hi])
        if self.gathers and self.gather_shadow:
            with torch.no_grad():
                self.exchange_fp32()
        self.gathers = []

    def gather_state(self, tensors=()) -> None:
        """COLLECTIVE: all-gather optimizer state buffers (flat, like the master) so every rank
        holds every piece (checkpoint save) -- and the fp32 master itself when the steps gather
        only the bf16 shadow."""
        if not self.shard:
            return
        if self.gather_shadow:
            tensors = [self.store.master] + list(tensors)
        for t in tensors:
            if t is None:
                continue
            for b in range(len(self.buckets)):
                self._gather_into(t, b).wait()

    def sum_(self, t: torch.Tensor) -> None:
        """In-place SUM all-reduce (sharded LAMB / LARS norms, global clip norm)."""
        if self.shard:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def bucket_ranges(self) -> list[tuple[int, int]]:
        return [(lo, hi) for lo, hi, _ in self.buckets]

    def optimizer_groups(self) -> list[list[int]]:
        """Consecutive bucket indices whose optimizer update is issued as ONE launch once all of
        them are reduced (``OPT_GROUPS`` = 4; 0 = one launch per bucket).  Buckets are
        contiguous flat ranges in launch order, so a group is one contiguous range.  Measured at one
        rank on RCCL: 30 per-bucket AdamW launches cost 0.4 ms/step more than one
        (profiles/r2_dp_overhead_1rank.txt); a few groups keep the update of the early buckets
        overlapped with the reduction of the last ones."""
        nb = len(self.buckets)
        g = OPT_GROUPS
        g = nb if g <= 0 else max(1, min(g, nb))
        return [list(range(nb * i // g, nb * (i + 1) // g)) for i in range(g)]

    def optimizer_pieces(self) -> list[list[tuple[int, int]]] | None:
        """Sharded: the owned pieces of each optimizer group (None when not sharded)."""
        if not self.shard:
            return None
        return [self.owned_pieces(grp) for grp in self.optimizer_groups()]

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
        for wk in self.works:
            left[gid[wk[0]]] += 1
        for b, w, to_div, lo, hi, staged, _ in self.works:
            w.wait()
            if to_div is not None:
                to_div.div_(self.world)
            if staged is not None:
                self.store.grad[lo:hi].copy_(staged)
            left[gid[b]] -= 1
            if on_bucket_done is not None and left[gid[b]] == 0:
                on_bucket_done(*ranges[gid[b]])
                for bb in groups[gid[b]]:  # sharded: the group's owned pieces are updated
                    self.gather(bb)
        if on_bucket_done is not None:  # a group without any reduction of its own (none today)
            for i, grp in enumerate(groups):
                if not any(gid[wk[0]] == i for wk in self.works):
                    on_bucket_done(*ranges[i])
                    for bb in grp:
                        self.gather(bb)
        self.works = []

    def stats(self) -> dict:
        sizes = [(hi - lo) * 4 / 2**20 for lo, hi, _ in self.buckets]
        return {"buckets": len(self.buckets), "bucket_mb_max": max(sizes) if sizes else 0.0,
                "bucket_mb_min": min(sizes) if sizes else 0.0,
                "mode": "zero1-reduce-scatter" if self.shard else "all-reduce",
                "reduce_dtype": "bf16" if self.reduce_dtype == torch.bfloat16 else "fp32",
                **({"gather_dtype": "bf16" if self.gather_shadow else "fp32"} if self.shard else {})}
