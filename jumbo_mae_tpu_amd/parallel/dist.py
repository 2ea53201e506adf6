"""Process-group setup: one process per GPU, torchrun env:// rendezvous, RCCL over xGMI.

Reference: the JAX runtime's implicit pmap SPMD world; ``jax.process_index``
/ ``process_count`` map to ``rank`` / ``world_size`` here because every GPU is its own process
(the reference's per-host batch split ``train_batch_size // process_count`` becomes a per-rank
split, dataset.py:129).
"""

from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str | None = None

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


_INFO = DistInfo()


def init_distributed(device: str | None = None, timeout_s: int = 1800) -> DistInfo:
    """Initialise from torchrun variables (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*).

    Backend ``nccl`` (== RCCL on ROCm) when GPUs are present, ``gloo`` otherwise.  The default
    collective timeout acts as the failure detector for a dead peer.
    """
    global _INFO
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() if device is None else device.startswith("cuda")
    if use_gpu:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    backend = None
    if (world > 1 or forced_group()) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        backend = "nccl" if use_gpu else "gloo"
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if use_gpu:
            kw["device_id"] = dev
            # RCCL's stream at high priority (JMAE_RCCL_HIPRI, default on): every compute kernel of the
            # step fills all 256 CUs, so at normal priority a collective's workgroups only get CUs
            # between kernels (1-rank trace: kernel union == kernel sum, no overlap at all); at high
            # priority the dispatcher places them as soon as a CU frees up and they run beside the
            # backward (union 4.1 ms below the sum; step 94.6 -> 93.2 ms, profiles/r2_dp_overhead_1rank.txt)
            if os.environ.get("JMAE_RCCL_HIPRI", "1") == "1":
                kw["pg_options"] = dist.ProcessGroupNCCL.Options(is_high_priority_stream=True)
        dist.init_process_group(**kw)
    elif dist.is_initialized():
        backend = dist.get_backend()
    _INFO = DistInfo(rank, world, local, dev, backend)
    return _INFO


def forced_group() -> bool:
    """``JMAE_FORCE_PG=1``: create the process group (and the gradient reducer) even at world size
    1.  Test/diagnostic switch: a 1-rank RCCL communicator runs every line of the data-parallel path
    (bucketed async all-reduce from the weight-gradient stream, per-bucket optimizer overlap,
    device barriers) on a one-GPU box, and AVG over one rank is the identity, so the step must equal
    the non-distributed step bit for bit (tests/test_rccl_gpu.py)."""
    return os.environ.get("JMAE_FORCE_PG", "0") == "1"


def info() -> DistInfo:
    return _INFO


def barrier():
    if dist.is_available() and dist.is_initialized():
        if _INFO.device.type == "cuda":
            dist.barrier(device_ids=[_INFO.device.index])
        else:
            dist.barrier()


def all_reduce_mean_(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place mean over ranks (pmean)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return t
    if dist.get_backend(group) == "nccl":
        dist.all_reduce(t, op=dist.ReduceOp.AVG, group=group)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.div_(dist.get_world_size(group))
    return t


def all_reduce_sum_(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place sum over ranks (psum)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def broadcast_(t: torch.Tensor, src: int = 0, group=None) -> torch.Tensor:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(t, src=src, group=group)
    return t


def all_reduce_max_scalar(x: float, device) -> float:
    t = torch.tensor([x], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_gather_object(obj) -> list:
    """Every rank's ``obj`` (picklable), in rank order, on every rank."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        out = [None] * dist.get_world_size()
        dist.all_gather_object(out, obj)
        return out
    return [obj]


def cleanup():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
