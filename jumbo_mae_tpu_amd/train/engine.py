"""Data-parallel train / eval step engine.

Reference: the pmap'd ``training_step`` / ``validation_step`` (/root/reference/src/pretraining.py:
125-167, finetuning.py:109-165).  One step = zero the flat grad buffer, run ``grad_accum``
micro-steps (forward, backward with the gradient writes fused into the backward kernels,
RCCL bucket all-reduce overlapped with the last micro-step's backward), one fused optimizer
pass.  Metrics stay on the device; they are averaged over ranks lazily when logged (the
reference pmean's them every step, CC3, which is a blocking host round trip we avoid).
"""

from __future__ import annotations


import torch

from ..ops.prims import join_wgrad_stream
from ..optim.flat import FlatOptimizer
from ..parallel.ddp import GradReducer
from ..utils.rng import RngStreams
from ..utils.trace import trace_range


class Trainer:
    def __init__(self, model, optimizer: FlatOptimizer, reducer: GradReducer | None = None,
                 rngs: RngStreams | None = None, grad_accum: int = 1, skip_nonfinite: bool = False):
        self.skip_nonfinite = skip_nonfinite
        self.skipped_steps = 0
        self.model = model
        self.opt = optimizer
        self.reducer = reducer
        self.rngs = rngs
        self.grad_accum = grad_accum
        # update each DP bucket right after its all-reduce (optimizer / reduction-tail overlap)
        self.overlap_optimizer = True
        self._planned = False
        self._comm_events = None  # (start, end) around the last step's reduction wait
        if reducer is not None and getattr(reducer, "shard", False):
            optimizer.attach_shard(reducer)  # ZeRO-1: owned pieces only, master all-gathered

    @property
    def store(self):
        return self.model.store

    def train_step(self, micro_batches) -> dict:
        """micro_batches: list (len grad_accum) of argument tuples for ``model.forward``."""
        self.host_prepare(micro_batches)
        metrics = self.device_step(micro_batches)
        if metrics is None:  # non-finite loss, update skipped
            return self._skipped
        metrics["learning_rate"] = self.host_finish()
        return metrics

    # The step in three parts (runtime/graph.py captures ``device_step`` in a HIP graph and
    # replays it; the host parts run before / after every replay):
    #   host_prepare -- host-drawn per-step values (schedule, Mixup / CutMix decisions) into the
    #                   step feeder's static device buffers;
    #   device_step  -- device work only: zero grads, forward / backward per micro-batch, gradient
    #                   reduction, optimizer kernels; returns device metric tensors;
    #   host_finish  -- host bookkeeping (optimizer count, weight-shadow version); returns the lr.
    def host_prepare(self, micro_batches) -> None:
        prep = getattr(self.model, "prepare_step", None)
        if prep is not None:
            for i, args in enumerate(micro_batches):
                prep(i, *args)
        self.opt.prepare()

    def device_step(self, micro_batches) -> dict | None:
        n = len(micro_batches)
        self.store.zero_grad()
        if self.reducer is not None:
            self.reducer.begin_step()
        metrics_acc = None
        rng = self.rngs.as_dict() if self.rngs is not None else {}
        for i, args in enumerate(micro_batches):
            if self.reducer is not None:
                self.reducer.set_sync(i == n - 1)
            self.model.micro_index = i
            with trace_range("fwd"):
                out = self.model(*args, rngs=rng, det=False)
            loss = out["loss"]
            with trace_range("bwd"):
                (loss / n).backward()
            m = {k: v.detach().float() for k, v in out.items()}
            metrics_acc = m if metrics_acc is None else {k: metrics_acc[k] + m[k] for k in m}
        join_wgrad_stream()  # weight-gradient GEMMs run on a side stream (ops/prims.py)
        self.store.flush_fresh()  # a store-mode gradient nobody wrote this step is zeroed
        split = (self.overlap_optimizer and self.reducer is not None and self.reducer.enabled
                 and self.opt.can_split() and not self.skip_nonfinite)
        if split and not self._planned:
            self.opt.plan_ranges(self.reducer.optimizer_ranges(), self.reducer.optimizer_pieces())
            self._planned = True
        if self.reducer is not None:
            with trace_range("allreduce_wait"):
                timed = self.reducer.enabled and self.store.grad.is_cuda and not torch.cuda.is_current_stream_capturing()
                if timed:
                    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    ev[0].record()
                self.reducer.set_sync(True)
                self.reducer.finish(self.opt.launch_range if split else None)
                if timed:
                    ev[1].record()
                    self._comm_events = ev
        metrics = {k: v / n for k, v in metrics_acc.items()}
        if self.skip_nonfinite:
            # opt-in guard (one host sync per step): drop the update of a step whose loss is
            # not finite instead of poisoning the weights / optimizer moments.
            # The decision is GLOBAL: a NaN on one rank has already reached every rank through the
            # gradient all-reduce, so every rank must skip together (a MAX over the ranks' flags)
            if self.nonfinite_anywhere(metrics_acc["loss"]):
                self.skipped_steps += 1
                metrics["learning_rate"] = self.opt.last_lr if hasattr(self.opt, "last_lr") else 0.0
                self._skipped = metrics
                return None
        with trace_range("optimizer"):
            if split:
                self.opt.launch_rest()
            else:
                self.opt.launch()
        if self.reducer is not None and self.reducer.shard:
            with trace_range("allgather_wait"):
                self.reducer.gather_all()    # groups not gathered during finish (monolithic update)
                self.reducer.wait_gathers()  # next forward reads the whole master / shadow
        return metrics

    def nonfinite_anywhere(self, loss: torch.Tensor) -> bool:
        """True when the loss is not finite on ANY rank of the data-parallel group."""
        bad = (~torch.isfinite(loss.detach().float())).float().reshape(1)
        r = self.reducer
        if r is not None and r.enabled:
            import torch.distributed as dist
            dist.all_reduce(bad, op=dist.ReduceOp.MAX, group=r.group)
        return bool(bad.item() > 0)

    def host_finish(self) -> float:
        return self.opt.finish()

    def comm_ms(self) -> float | None:
        """GPU time the last step spent behind the data-parallel reduction after its backward was
        queued (the exposed communication, including overlapped bucket updates); None without a
        reducer.  Synchronises on that step's end event: call it at log intervals only."""
        if self._comm_events is None:
            return None
        e0, e1 = self._comm_events
        e1.synchronize()
        return e0.elapsed_time(e1)

    @torch.no_grad()
    def eval_step(self, args) -> dict:
        rng = self.rngs.as_dict() if self.rngs is not None else {}
        return self.model.evaluate(*args, rngs=rng)
