"""Collective timing helpers shared by ``tools/allreduce_bench.py`` (node sweeps) and ``bench.py``
(self-calibration of the first multi-GPU run: the real bucket sizes of the step's reducer plan,
timed on the real process group after the timed steps).

Bus bandwidth convention of nccl-tests: all-reduce busbw = bytes / t * 2 (n - 1) / n; reduce-scatter
and all-gather busbw = bytes / t * (n - 1) / n (bytes = the full, unsharded buffer).  The rows are
the ``collective_sweep`` records ``tools/dp_exposure_model.py --sweep`` reads."""

from __future__ import annotations

import time

import torch
import torch.distributed as dist


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def time_collective(fn, iters: int, warmup: int, dev, group=None) -> float:
    """Mean seconds per call of ``fn`` (issued back to back), MAX over the ranks."""
    for _ in range(warmup):
        fn()
    _sync(dev)
    dist.barrier(group=group)
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    _sync(dev)
    dt = (time.perf_counter() - t0) / iters
    t = torch.tensor([dt], dtype=torch.float64, device=dev if dev.type == "cuda" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def sweep(sizes_bytes, dtype: torch.dtype, iters: int, warmup: int, ops, dev, group=None) -> list[dict]:
    """One row per message size (bytes, rounded to a multiple of world elements)."""
    n = dist.get_world_size(group)
    esz = torch.tensor([], dtype=dtype).element_size()
    rows = []
    for nb in sizes_bytes:
        numel = max(n, int(nb) // esz // n * n)
        nbytes = numel * esz
        buf = torch.ones(numel, dtype=dtype, device=dev)
        res = {"size_mb": round(nbytes / 2**20, 3), "bytes": nbytes, "dtype": str(dtype).replace("torch.", ""),
               "world": n}
        if "allreduce" in ops:
            t = time_collective(lambda: dist.all_reduce(buf, group=group), iters, warmup, dev, group)
            res["allreduce_ms"] = t * 1e3
            res["allreduce_algbw_GBs"] = nbytes / t / 1e9
            res["allreduce_busbw_GBs"] = nbytes / t / 1e9 * 2 * (n - 1) / n
        if "reduce_scatter" in ops:
            out = torch.empty(numel // n, dtype=dtype, device=dev)
            t = time_collective(lambda: dist.reduce_scatter_tensor(out, buf, group=group), iters, warmup, dev, group)
            res["reduce_scatter_ms"] = t * 1e3
            res["reduce_scatter_busbw_GBs"] = nbytes / t / 1e9 * (n - 1) / n
        if "all_gather" in ops:
            part = torch.ones(numel // n, dtype=dtype, device=dev)
            t = time_collective(lambda: dist.all_gather_into_tensor(buf, part, group=group), iters, warmup, dev,
                                group)
            res["all_gather_ms"] = t * 1e3
            res["all_gather_busbw_GBs"] = nbytes / t / 1e9 * (n - 1) / n
        rows.append(res)
        del buf
    return rows


def plan_sizes(reducer) -> list[int]:
    """Distinct collective message sizes (bytes) of a GradReducer's bucket plan, ascending."""
    esz = 2 if reducer.reduce_dtype == torch.bfloat16 else 4
    return sorted({(hi - lo) * esz for lo, hi, _ in reducer.buckets})


def calibrate(reducer, dev, iters: int = 5, warmup: int = 2) -> list[dict]:
    """Time one collective per distinct bucket size of the reducer's real plan (the collectives the
    step issues: all-reduce, or reduce-scatter + all-gather for ZeRO-1)."""
    ops = ("reduce_scatter", "all_gather") if reducer.shard else ("allreduce",)
    return sweep(plan_sizes(reducer), reducer.reduce_dtype, iters, warmup, ops, dev, reducer.group)
