"""Fixed 2-D sin-cos position table.

Parity: ``fixed_sincos2d_embeddings`` (/root/reference/src/utils.py:114-121).  Note the
reference uses ``linspace(0, 1, dim//4)`` (endpoint included) for the frequency exponent,
not MAE's ``arange/(dim/4)``; the output is ``(ncols, nrows, dim)`` laid out as
``[sin x, cos x, sin y, cos y]`` where x runs along the second (width) axis.
The table is built once on the host in float32 (constant, never a parameter).
"""

from __future__ import annotations

import functools

import numpy as np
import torch


@functools.lru_cache(maxsize=32)
def _sincos2d_np(ncols: int, nrows: int, dim: int) -> np.ndarray:
    d4 = dim // 4
    # float32 end-to-end like jnp (default dtype float32 on TPU).
    freqs = (1.0 / (np.float32(10000.0) ** np.linspace(0, 1, d4, dtype=np.float32))).astype(np.float32)
    x = np.outer(np.arange(0, nrows, dtype=np.float32), freqs).astype(np.float32)
    y = np.outer(np.arange(0, ncols, dtype=np.float32), freqs).astype(np.float32)
    x = np.broadcast_to(x[None, :, :], (ncols, nrows, d4))
    y = np.broadcast_to(y[:, None, :], (ncols, nrows, d4))
    return np.concatenate((np.sin(x), np.cos(x), np.sin(y), np.cos(y)), axis=2).astype(np.float32)


def fixed_sincos2d_embeddings(ncols: int, nrows: int, dim: int, device=None) -> torch.Tensor:
    return torch.from_numpy(_sincos2d_np(ncols, nrows, dim).copy()).to(device)
