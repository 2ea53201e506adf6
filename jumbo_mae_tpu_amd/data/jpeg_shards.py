"""Write webdataset-style tar shards of real JPEG images (``<key>.jpg`` + ``<key>.cls``).

No dataset is reachable offline, so the driver tests on the GPU (tests/test_drivers_gpu.py) and the
input-pipeline rate benchmark (tools/data_rate_bench.py) read shards written here: JPEG files
encoded by PIL at ImageNet-like sizes (long side 375-500 px, quality 90, ~40-110 KB), through the
same tar reader, decoder, transforms and collate as ImageNet shards would go
(/root/reference/src/dataset.py:56-82, :100-161).  The pictures are class-conditioned so a
classifier can learn them: a smooth two-colour gradient whose hue is set by the label, a few
ellipses and mild noise.

    python -m jumbo_mae_tpu_amd.data.jpeg_shards <dir> --shards 4 --per-shard 256 --classes 10
"""

from __future__ import annotations

import argparse
import colorsys
import io
import os
import tarfile

import numpy as np


def synth_image(rng: np.random.Generator, label: int, classes: int, size: tuple[int, int]) -> np.ndarray:
    """H x W x 3 uint8 picture of class ``label``."""
    w, h = size
    hue = (label + 0.3 * rng.random()) / max(classes, 1)
    c0 = np.array(colorsys.hsv_to_rgb(hue, 0.8, 0.9)) * 255
    c1 = np.array(colorsys.hsv_to_rgb((hue + 0.5) % 1.0, 0.5, 0.35)) * 255
    ang = rng.random() * 2 * np.pi
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    t = (np.cos(ang) * xx / w + np.sin(ang) * yy / h)
    t = (t - t.min()) / max(float(np.ptp(t)), 1e-6)
    img = c0[None, None, :] * (1 - t[..., None]) + c1[None, None, :] * t[..., None]
    for _ in range(int(rng.integers(2, 6))):
        cx, cy = rng.random() * w, rng.random() * h
        rx, ry = (0.05 + 0.2 * rng.random()) * w, (0.05 + 0.2 * rng.random()) * h
        m = ((xx - cx) / rx) ** 2 + ((yy - cy) / ry) ** 2 <= 1.0
        img[m] = rng.integers(0, 256, 3)
    img += rng.normal(0.0, 6.0, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def jpeg_bytes(arr: np.ndarray, quality: int = 90) -> bytes:
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, format="JPEG", quality=quality)
    return buf.getvalue()


def write_shards(out_dir: str, shards: int = 4, per_shard: int = 256, classes: int = 10, seed: int = 0,
                 prefix: str = "train", quality: int = 90) -> str:
    """Writes ``{prefix}-{i:06d}.tar`` and returns the brace spec ``{prefix}-{000000..N-1}.tar``."""
    os.makedirs(out_dir, exist_ok=True)
    rng = np.random.default_rng(seed)
    for s in range(shards):
        path = os.path.join(out_dir, f"{prefix}-{s:06d}.tar")
        with tarfile.open(path + ".tmp", "w", format=tarfile.USTAR_FORMAT) as tf:
            for i in range(per_shard):
                label = int(rng.integers(0, classes))
                long_side = int(rng.integers(375, 501))
                short_side = int(long_side * (0.66 + 0.09 * rng.random()))
                size = (long_side, short_side) if rng.random() < 0.75 else (short_side, long_side)
                key = f"{prefix}_{s:06d}_{i:06d}"
                for name, data in ((f"{key}.jpg", jpeg_bytes(synth_image(rng, label, classes, size), quality)),
                                   (f"{key}.cls", str(label).encode())):
                    ti = tarfile.TarInfo(name)
                    ti.size = len(data)
                    tf.addfile(ti, io.BytesIO(data))
        os.replace(path + ".tmp", path)
    return os.path.join(out_dir, f"{prefix}-{{{0:06d}..{shards - 1:06d}}}.tar")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir")
    ap.add_argument("--shards", type=int, default=4)
    ap.add_argument("--per-shard", type=int, default=256)
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--prefix", default="train")
    a = ap.parse_args(argv)
    print(write_shards(a.out_dir, a.shards, a.per_shard, a.classes, a.seed, a.prefix))


if __name__ == "__main__":
    main()
