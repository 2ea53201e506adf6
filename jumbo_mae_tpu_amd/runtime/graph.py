"""HIP-graph capture and replay of a whole train step (forward, backward, optimizer).

MI355X-native replacement for a tracing compiler's launch-overhead removal: the step is captured
once with ``torch.cuda.CUDAGraph`` (hipGraph on ROCm) and replayed every iteration, so ~800-1500
kernel launches cost one graph launch and the GPU never waits for Python between kernels.

What makes the step capturable (engine.Trainer splits it into host / device parts):
* inputs: micro-batches are copied into static device tensors before each replay;
* host-drawn values (learning-rate schedule, bias corrections, Mixup / CutMix decisions and
  permutations) reach the step only through the step feeder's static device buffers
  (runtime/feeder.py), written by ``Trainer.host_prepare`` outside the graph;
* device RNG (MAE masking noise, droppath / dropout masks) uses the per-stream device
  generators, registered with the graph so every replay advances their Philox offsets;
* the step contains no host synchronisation (``--skip-nonfinite`` is refused in graph mode);
* parameter gradients, optimizer moments, master weights and the bf16 shadow are persistent
  buffers of the flat ParamStore -- the captured kernels update them in place.
Scope: single-process steps (no DP reducer): RCCL collectives are not captured here.
"""

from __future__ import annotations


import torch


def _state_tensors(trainer) -> list[torch.Tensor]:
    """Persistent tensors a step mutates (restored after warm-up / capture with ``restore``)."""
    ts = [trainer.store.master]
    for k in ("mu", "nu", "trace"):
        v = getattr(trainer.opt, k, None)
        if v is not None:
            ts.append(v)
    head = getattr(trainer.model, "head", None)
    for k in ("running_mean", "running_var"):
        v = getattr(head, k, None) if head is not None else None
        if isinstance(v, torch.Tensor):
            ts.append(v)
    return ts


class GraphedTrainStep:
    """``restore=True`` (training drivers): the warm-up steps are undone afterwards --
    weights, optimizer moments, BatchNorm statistics and the optimizer count are put back, so the
    first replay is the run's first real step (device RNG streams simply continue)."""

    def __init__(self, trainer, example_micro_batches, warmup: int = 3, restore: bool = False):
        if trainer.reducer is not None and trainer.reducer.enabled:
            raise ValueError("HIP-graph step capture is single-process (no DP reducer)")
        if trainer.skip_nonfinite:
            raise ValueError("--skip-nonfinite needs a host sync per step; not capturable")
        self.tr = trainer
        # Store-mode gradients in captured steps (allow_store=False would zero-then-accumulate).  A
        # hipMemsetAsync captured into the graph left the small store-mode gradients as garbage on
        # replay; those zero fills are kernels now (csrc/elementwise.hip jm_zero_f32) and the replay
        # matches the eager step bit for bit (tests/test_graph_gpu.py::
        # test_graphed_grads_match_eager_production_routing, tools/graph_grad_diag.py).
        trainer.store.allow_store = True
        self.static = [tuple(t.clone() for t in mb) for mb in example_micro_batches]
        snap = None
        if restore:
            snap = ([t.clone() for t in _state_tensors(trainer)], trainer.opt.count, trainer.opt.last_lr)
        # warm up eagerly on a side stream (allocator pools, lazy weight copies, hipBLASLt plans)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                trainer.train_step(self.static)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        if trainer.rngs is not None:
            for gen in trainer.rngs.gens.values():
                self.graph.register_generator_state(gen)
        trainer.host_prepare(self.static)
        with torch.cuda.graph(self.graph):  # recorded, not executed: no host_finish for it
            self.out = trainer.device_step(self.static)
        self.replays = 0
        if snap is not None:
            torch.cuda.synchronize()
            for dst, src in zip(_state_tensors(trainer), snap[0]):
                dst.copy_(src)
            trainer.opt.count, trainer.opt.last_lr = snap[1], snap[2]
            trainer.store.sync_shadow()
            torch.cuda.synchronize()

    def __call__(self, micro_batches) -> dict:
        for st, mb in zip(self.static, micro_batches):
            for dst, src in zip(st, mb):
                if dst.data_ptr() != src.data_ptr():
                    dst.copy_(src, non_blocking=True)
        self.tr.host_prepare(self.static)
        self.graph.replay()
        self.replays += 1
        lr = self.tr.host_finish()
        m = {k: v.clone() for k, v in self.out.items()}
        m["learning_rate"] = lr
        return m


class StepRunner:
    """``trainer.train_step`` or, with ``hip_graph``, a GraphedTrainStep built on the first call
    (drivers: ``--hip-graph``)."""

    def __init__(self, trainer, hip_graph: bool = False):
        self.tr = trainer
        self.hip_graph = hip_graph
        self.graphed = None

    def __call__(self, micro_batches) -> dict:
        if not self.hip_graph:
            return self.tr.train_step(micro_batches)
        if self.graphed is None:
            self.graphed = GraphedTrainStep(self.tr, micro_batches, restore=True)
        return self.graphed(micro_batches)
