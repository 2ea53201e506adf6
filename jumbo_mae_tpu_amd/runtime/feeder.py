"""Per-step host values (learning rate, bias corrections, Mixup / CutMix decisions, permutations)
delivered to STATIC device buffers.

Every value a train step needs from the host goes through ``StepFeeder.put(name, values)``: the
values are written into a slot of a small ring of pinned host buffers and copied (async, on the
current stream) into one device tensor per name whose address never changes.  Kernels and torch
ops of the step read only those device tensors, so the step itself has no host inputs and can be
captured once into a HIP graph and replayed (runtime/graph.py); the puts run before each replay,
outside the graph.  A ring slot is reused only after the copy that read it has completed (an
event per slot), so the host may run several steps ahead of the GPU without overwriting values
an in-flight copy still has to read.
"""

from __future__ import annotations

import torch

_RING = 4


class StepFeeder:
    def __init__(self, device):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self._dev: dict[str, torch.Tensor] = {}
        self._host: dict[str, list[torch.Tensor]] = {}
        self._events: dict[str, list] = {}
        self._slot: dict[str, int] = {}

    def buffer(self, name: str) -> torch.Tensor:
        return self._dev[name]

    def put(self, name: str, values, dtype=torch.float32) -> torch.Tensor:
        """Copy ``values`` (sequence / numpy / CPU tensor) into the static device buffer ``name``."""
        src = torch.as_tensor(values, dtype=dtype).reshape(-1)
        if name not in self._dev:
            self._dev[name] = torch.empty(src.numel(), dtype=dtype, device=self.device)
            if self.cuda:
                self._host[name] = [torch.empty(src.numel(), dtype=dtype, pin_memory=True) for _ in range(_RING)]
                self._events[name] = [None] * _RING
                self._slot[name] = 0
        dst = self._dev[name]
        if dst.numel() != src.numel() or dst.dtype != dtype:
            raise ValueError(f"feeder buffer {name}: shape/dtype changed ({dst.numel()} -> {src.numel()})")
        if not self.cuda:
            dst.copy_(src)
            return dst
        i = self._slot[name]
        self._slot[name] = (i + 1) % _RING
        ev = self._events[name][i]
        if ev is not None:
            ev.synchronize()  # the copy that last read this slot has run
        host = self._host[name][i]
        host.copy_(src)
        dst.copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._events[name][i] = ev
        return dst


_FEEDERS: dict[str, StepFeeder] = {}


def feeder(device) -> StepFeeder:
    """Process-wide feeder per device."""
    key = str(torch.device(device))
    if key not in _FEEDERS:
        _FEEDERS[key] = StepFeeder(device)
    return _FEEDERS[key]
