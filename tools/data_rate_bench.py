"""Input-pipeline rate: JPEG tar shards -> decode -> RandomResizedCrop(0.2-1, bicubic) + flip (+
RandAugment / random erasing for finetuning) -> collate -> (optionally) pinned H2D, per loader
worker count.  The reference feeds each TPU host from 40 loader workers with pillow-simd
(/root/reference/src/dataset.py:100-161, /root/reference/scripts/setup.sh:31-34); this measures how
many workers of THIS loader (data/loader.py, native tar reader, PIL) one MI355X needs at its
training rate.  Shards are written with real JPEG files at ImageNet-like sizes
(data/jpeg_shards.py) on first use.

    python tools/data_rate_bench.py [--workers 1,2,4,8] [--mode pretrain|finetune] [--batch 256]
                                    [--h2d] [--device-augment]

Prints one JSON line per worker count: steady-state images/s of the loader (after draining what
the workers prefetched), per worker, and with ``--h2d`` the rate through the DevicePrefetcher
(pinned batches copied to the GPU on a side stream; with ``--device-augment`` also resized there)
plus the host->device copy bandwidth."""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jumbo_mae_tpu_amd.data.jpeg_shards import write_shards  # noqa: E402
from jumbo_mae_tpu_amd.data.loader import create_dataloaders  # noqa: E402


def loader_args(spec: str, mode: str, batch: int, workers: int) -> SimpleNamespace:
    ft = mode == "finetune"
    return SimpleNamespace(
        random_crop="rrc", image_size=224, auto_augment="rand-m9-mstd0.5-inc1" if ft else "none",
        color_jitter=0.0, random_erasing=0.25 if ft else 0.0, test_crop_ratio=0.875,
        train_dataset_shards=spec, valid_dataset_shards=None, mode=mode, train_batch_size=batch, grad_accum=1,
        augment_repeats=1, shuffle_seed=0, train_loader_workers=workers, valid_batch_size=batch,
        valid_loader_workers=0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/tmp/jmae_jpeg_shards")
    ap.add_argument("--shards", type=int, default=16)
    ap.add_argument("--per-shard", type=int, default=256)
    ap.add_argument("--workers", default="1,2,4,8")
    ap.add_argument("--mode", default="pretrain", choices=["pretrain", "finetune"])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--h2d", action="store_true", help="also through the DevicePrefetcher onto cuda:0")
    ap.add_argument("--device-augment", action="store_true",
                    help="workers decode + ship crop windows; resize / flip on the GPU (csrc/augment.hip)")
    a = ap.parse_args()
    spec = os.path.join(a.dir, f"train-{{000000..{a.shards - 1:06d}}}.tar")
    if not os.path.exists(os.path.join(a.dir, f"train-{a.shards - 1:06d}.tar")):
        t0 = time.time()
        write_shards(a.dir, a.shards, a.per_shard, classes=1000, seed=0)
        print(f"[data] wrote {a.shards} x {a.per_shard} JPEGs in {time.time() - t0:.1f}s", file=sys.stderr)
    sizes = [os.path.getsize(os.path.join(a.dir, f"train-{i:06d}.tar")) for i in range(a.shards)]
    mean_kb = sum(sizes) / (a.shards * a.per_shard) / 1024
    def steady(it, nw, batch):
        """Steady-state images/s: first drain what the workers prefetched before the clock starts
        (up to nw x prefetch_factor batches), then time 6x that many batches (a backlog refilled
        while draining is then at most a sixth of the timed batches)."""
        for _ in range(nw * 4 + 2):
            last = next(it)
        k = 6 * 4 * max(nw, 1)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            last = next(it)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        return k * batch / (time.perf_counter() - t0), last

    for nw in [int(x) for x in a.workers.split(",")]:
        dl, _ = create_dataloaders(loader_args(spec, a.mode, a.batch, nw), device_augment=a.device_augment)
        rate, b = steady(iter(dl), nw, a.batch)
        out = {"mode": a.mode, "device_augment": a.device_augment, "workers": nw, "images_per_sec": round(rate, 1),
               "per_worker": round(rate / max(nw, 1), 1), "batch": a.batch, "jpeg_kb": round(mean_kb, 1),
               "cpus": os.cpu_count()}
        if a.device_augment:
            out["window_kb_per_image"] = round(b.src.numel() / a.batch / 1024, 1)
        del dl
        if a.h2d and torch.cuda.is_available():
            from jumbo_mae_tpu_amd.train.common import DevicePrefetcher
            dev = torch.device("cuda:0")
            dl, _ = create_dataloaders(loader_args(spec, a.mode, a.batch, nw), device_augment=a.device_augment)
            rate, x = steady(DevicePrefetcher(dl, dev), nw, a.batch)
            out["prefetcher_images_per_sec"] = round(rate, 1)
            out["device_shape"] = list((x[0] if isinstance(x, (list, tuple)) else x).shape)
            host = (x[0] if isinstance(x, (list, tuple)) else x).cpu().pin_memory()
            buf = torch.empty_like(host, device=dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                buf.copy_(host, non_blocking=True)
            torch.cuda.synchronize()
            out["h2d_gb_per_sec"] = round(20 * host.numel() / (time.perf_counter() - t0) / 1e9, 2)
            del dl
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
