"""Bytes the device augment ships and the device scratch it allocates, per batch.

The device augment (data/loader.py DeviceRRCParams / collate_packed, csrc/augment.hip) ships each
image's RandomResizedCrop window plus the bicubic filter margin, not the resized 224 x 224 result,
and the horizontal pass writes a [rows x 224 x 3] scratch per image on the prefetch stream.  This
tool draws crops exactly as the loader workers do, on images of the ImageNet-like size distribution
of data/jpeg_shards.py (long side 375-500 px, 3:2-4:3 aspect, 3/4 landscape), and reports per batch:

* H2D bytes (windows + descriptors) against the uint8 224 x 224 x 3 images the host path ships;
* the horizontal-pass scratch (``PackedImages.tmp_bytes``);
* on a GPU (``--gpu``): the allocator's peak during ``unpack_on_device`` above the memory held
  before it (the transient footprint: windows + descriptors + scratch + output).

    python tools/augment_bytes.py [--batch 512] [--batches 8] [--gpu] [--json out.json]
"""

from __future__ import annotations

import argparse
import json
import os
import random
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def draw_sizes(rng: np.random.Generator, n: int):
    out = []
    for _ in range(n):
        long_side = int(rng.integers(375, 501))
        short_side = int(long_side * (0.66 + 0.09 * rng.random()))
        out.append((long_side, short_side) if rng.random() < 0.75 else (short_side, long_side))
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--json", default="")
    a = ap.parse_args(argv)
    from PIL import Image

    from jumbo_mae_tpu_amd.data.loader import DeviceRRCParams, collate_packed

    random.seed(a.seed)
    import torch
    torch.manual_seed(a.seed)
    rng = np.random.default_rng(a.seed)
    tf = DeviceRRCParams(a.size)
    host_img = a.batch * 3 * a.size * a.size
    rows = []
    for bi in range(a.batches):
        items = [tf(Image.new("RGB", wh)) for wh in draw_sizes(rng, a.batch)]
        fallback = sum(int(d[5] == a.size and d[6] == a.size and d[9] == a.size) for _, d in items)
        p = collate_packed(items, size=a.size)
        h2d = p.src.numel() * p.src.element_size() + p.tab.numel() * p.tab.element_size()
        r = {"batch": bi, "h2d_bytes": h2d, "h2d_over_host_images": h2d / host_img, "tmp_bytes": p.tmp_bytes,
             "rows_max": p.rows_max, "fallback_crops": fallback}
        if a.gpu:
            from jumbo_mae_tpu_amd.data.loader import unpack_on_device
            dev = torch.device("cuda")
            torch.cuda.synchronize()
            base = torch.cuda.memory_allocated(dev)
            torch.cuda.reset_peak_memory_stats(dev)
            out = unpack_on_device(p, dev)
            torch.cuda.synchronize()
            r["gpu_transient_peak_bytes"] = torch.cuda.max_memory_allocated(dev) - base
            r["output_bytes"] = out.numel()
            del out
            torch.cuda.empty_cache()
        rows.append(r)
        print(json.dumps(r), flush=True)
    mb = 2.0 ** 20
    summ = {"batch": a.batch, "batches": a.batches, "host_images_mb": host_img / mb,
            "h2d_mb_mean": float(np.mean([r["h2d_bytes"] for r in rows])) / mb,
            "h2d_mb_max": max(r["h2d_bytes"] for r in rows) / mb,
            "h2d_over_host_images_mean": float(np.mean([r["h2d_over_host_images"] for r in rows])),
            "tmp_mb_mean": float(np.mean([r["tmp_bytes"] for r in rows])) / mb,
            "tmp_mb_max": max(r["tmp_bytes"] for r in rows) / mb,
            "fallback_crop_frac": sum(r["fallback_crops"] for r in rows) / (a.batch * a.batches)}
    if a.gpu:
        summ["gpu_transient_peak_mb_max"] = max(r["gpu_transient_peak_bytes"] for r in rows) / mb
    print(json.dumps({"summary": summ}), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"summary": summ, "rows": rows}, f, indent=1)
    return summ


if __name__ == "__main__":
    main()
