"""Collective bandwidth sweep for the data-parallel gradient path.

    torchrun --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29511 \
        tools/allreduce_bench.py --sizes-mb 1,4,16,64,128,256,512 --dtype fp32
    python tools/allreduce_bench.py --cpu --world 2          # gloo rehearsal on the host

For each message size it times ``all_reduce`` (and optionally reduce_scatter / all_gather), one
process per GPU over RCCL (backend ``nccl``), and reports

    algbw = bytes / t            busbw = algbw * 2 (n - 1) / n      (ring all-reduce, nccl-tests)

An 8 x MI355X node is fully connected by xGMI (7 links per GPU, ~153 GB/s each): a single ring is
per-link bound (~153 GB/s busbw) while RCCL's multi-channel rings can use all 7 links.  The bucket
size of ``parallel.ddp.GradReducer`` (``--bucket-mb``, default 64) should sit on the plateau of this
curve; the sweep also reports the modelled exposed time of the ViT-L gradient all-reduce
(1.62 GB fp32, of which the 302 MB shared jumbo-MLP gradient is the tail that cannot overlap).

Rank 0 prints a table and one JSON line (``{"collective_sweep": [...]}``); times are the max over
ranks of the per-iteration mean.  ``model.recommended_bucket_mb`` is the smallest swept size that
reaches 90 % of the best all-reduce bus bandwidth: pass it as ``--bucket-mb`` (bench.py / the
training CLI) -- larger buckets only delay the first reduction behind the backward pass.

RCCL knobs worth sweeping with this tool (environment, one run per setting; the defaults are what
bench.py uses): ``NCCL_MIN_NCHANNELS`` / ``NCCL_MAX_NCHANNELS`` (channels = rings in flight; on
8 fully connected xGMI GPUs enough channels are needed to drive all 7 links of a GPU),
``NCCL_PROTO`` (``Simple`` for large buckets, ``LL128`` / ``LL`` for small ones), ``NCCL_ALGO``
(``Ring`` / ``Tree``).  Keep ``HSA_ENABLE_IPC_MODE_LEGACY=0`` exported (dmabuf IPC).
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

DTYPES = {"fp32": torch.float32, "bf16": torch.bfloat16}
VIT_L_GRAD_BYTES = 404_901_632 * 4
VIT_L_JUMBO_TAIL_BYTES = 75_512_832 * 4


def sweep(sizes_mb, dtype: torch.dtype, iters: int, warmup: int, ops, dev) -> list[dict]:
    from jumbo_mae_tpu_amd.parallel.collbench import sweep as _sweep
    return _sweep([mb * 2**20 for mb in sizes_mb], dtype, iters, warmup, ops, dev)


def model_exposed(rows: list[dict]) -> dict:
    """ViT-L gradient all-reduce time at the best measured all-reduce bus bandwidth, and the part
    that the backward pass cannot hide (the shared jumbo-MLP gradient, final after layer 0)."""
    ar = [r for r in rows if "allreduce_busbw_GBs" in r]
    if not ar:
        return {}
    best = max(ar, key=lambda r: r["allreduce_busbw_GBs"])
    n = best["world"]
    bw = best["allreduce_busbw_GBs"] * 1e9 / (2 * (n - 1) / n) if n > 1 else float("inf")
    rec = min((r for r in ar if r["allreduce_busbw_GBs"] >= 0.9 * best["allreduce_busbw_GBs"]),
              key=lambda r: r["size_mb"])
    return {"best_busbw_GBs": best["allreduce_busbw_GBs"], "best_size_mb": best["size_mb"],
            "recommended_bucket_mb": rec["size_mb"],
            "vit_l_grad_allreduce_ms": VIT_L_GRAD_BYTES / bw * 1e3,
            "vit_l_jumbo_tail_ms": VIT_L_JUMBO_TAIL_BYTES / bw * 1e3}


def run(args, rank: int | None = None, world: int | None = None, port: int | None = None):
    if rank is not None:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from jumbo_mae_tpu_amd.parallel import dist as pdist

    info = pdist.init_distributed("cpu" if args.cpu else None)
    if not dist.is_initialized():  # world 1: a trivial group so the sweep still runs
        dist.init_process_group("gloo" if info.device.type == "cpu" else "nccl", rank=0, world_size=1,
                                init_method=f"tcp://127.0.0.1:{args.port}")
    sizes = [float(s) for s in args.sizes_mb.split(",")]
    rows = sweep(sizes, DTYPES[args.dtype], args.iters, args.warmup, args.ops.split(","), info.device)
    if dist.get_rank() == 0:
        for r in rows:
            print("  ".join(f"{k}={v:.3f}" if isinstance(v, float) else f"{k}={v}" for k, v in r.items()),
                  flush=True)
        out = {"collective_sweep": rows, "model": model_exposed(rows), "backend": dist.get_backend()}
        print(json.dumps(out), flush=True)
        if args.json:
            with open(args.json, "w") as f:
                json.dump(out, f, indent=1)
    dist.barrier()
    dist.destroy_process_group()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="1,4,16,64,128,256")
    ap.add_argument("--dtype", default="fp32", choices=sorted(DTYPES))
    ap.add_argument("--ops", default="allreduce,reduce_scatter,all_gather")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu", action="store_true", help="gloo on the host (rehearsal)")
    ap.add_argument("--world", type=int, default=0, help="spawn this many local ranks (with --cpu)")
    ap.add_argument("--port", type=int, default=29517)
    ap.add_argument("--json", default="")
    args = ap.parse_args(argv)
    if args.world > 1:
        if not args.cpu:
            raise SystemExit("--world spawns host ranks: use torchrun for GPU ranks")
        mp.spawn(_spawn_entry, args=(args, args.world, args.port), nprocs=args.world, join=True)
        return
    run(args)


def _spawn_entry(rank, args, world, port):
    run(args, rank, world, port)


if __name__ == "__main__":
    main()
