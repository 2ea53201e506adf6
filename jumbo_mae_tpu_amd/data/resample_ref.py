"""NumPy mirror of the device augment kernels (csrc/augment.hip): Pillow's bicubic resample
(Resample.c: precompute_coeffs, 22-bit fixed-point taps, horizontal pass into 8-bit rows, vertical
pass, clip8) evaluated on a crop window in the original image's coordinates, then the flip.  It is
bit-exact to ``PIL.Image.resize(size, BICUBIC, box)`` (tests/test_data.py checks that against PIL)
and is the CPU oracle of the GPU kernels (tests/test_augment_gpu.py)."""

from __future__ import annotations

import math

import numpy as np

PB = 22  # Pillow PRECISION_BITS


def _bicubic(x: float) -> float:
    a = -0.5
    if x < 0.0:
        x = -x
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def coeffs(in_size: int, in0: float, in1: float, out_size: int):
    """Per output coordinate: (first input index, fixed-point taps) as Pillow computes them."""
    in0, in1 = float(np.float32(in0)), float(np.float32(in1))
    scale = float(np.float32(in1 - in0)) / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    ss = 1.0 / filterscale
    out = []
    for xx in range(out_size):
        center = in0 + (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [_bicubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for v in w:
            ww += v
        if ww != 0.0:
            w = [v / ww for v in w]
        k = [int(-0.5 + v * (1 << PB)) if v < 0 else int(0.5 + v * (1 << PB)) for v in w]
        out.append((xmin, np.array(k, dtype=np.int64)))
    return out


def _clip8(s: np.ndarray) -> np.ndarray:
    return np.where(s >= (1 << PB << 8), 255, np.where(s <= 0, 0, s >> PB)).astype(np.uint8)


def resize_window(win: np.ndarray, desc, size: int) -> np.ndarray:
    """One descriptor (csrc/augment.hip layout) -> uint8 [3, size, size]."""
    _, wh, ww, y0, x0, H, W, i, j, ch, cw, flip = (int(v) for v in desc[:12])
    a = win.reshape(wh, ww, 3).astype(np.int64)
    cv = coeffs(H, i, i + ch, size)
    chh = coeffs(W, j, j + cw, size)
    first = cv[0][0]
    last = cv[-1][0] + len(cv[-1][1])
    tmp = np.zeros((last - first, size, 3), np.int64)
    for xx, (xmin, k) in enumerate(chh):
        s = (1 << (PB - 1)) + (a[first - y0:last - y0, xmin - x0:xmin - x0 + len(k), :] * k[None, :, None]).sum(1)
        tmp[:, xx, :] = _clip8(s)
    out = np.zeros((size, size, 3), np.uint8)
    for yy, (ymin, k) in enumerate(cv):
        s = (1 << (PB - 1)) + (tmp[ymin - first:ymin - first + len(k)] * k[:, None, None]).sum(0)
        out[yy] = _clip8(s)
    if flip:
        out = out[:, ::-1]
    return np.ascontiguousarray(out.transpose(2, 0, 1))


def unpack_packed(p) -> np.ndarray:
    """A ``data.loader.PackedImages`` batch -> uint8 [B, 3, S, S] (the kernels' result)."""
    src, tab = p.src.numpy(), p.tab.numpy()
    outs = []
    for d in tab:
        n = int(d[1]) * int(d[2]) * 3
        outs.append(resize_window(src[int(d[0]):int(d[0]) + n], d, p.size))
    return np.stack(outs)


def taps(c: int, out: int) -> int:
    return math.ceil(2.0 * max(c / out, 1.0)) * 2 + 1
