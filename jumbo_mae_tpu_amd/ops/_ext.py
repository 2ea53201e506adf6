"""Loader for the in-tree HIP extension (``jumbo_mae_tpu_amd/_C*.so``).

The extension is built by ``jumbo_mae_tpu_amd/csrc/build.py`` (hipcc --offload-arch=gfx950,
no hipify, no CUDA shims).  On a GPU box the fused kernels are *required*: if the shared
object is missing we fail loudly instead of silently falling back to eager PyTorch
(set ``JMAE_ALLOW_TORCH_FALLBACK=1`` to opt into the slow path explicitly).

``JMAE_EXT=debug`` loads ``_C_debug`` (soft device checks, ``debug_lines()``) and ``JMAE_EXT=asan``
loads ``_C_asan`` (host code under AddressSanitizer) instead; both are built with
``python -m jumbo_mae_tpu_amd.csrc.build --variant debug|asan``.
"""

from __future__ import annotations

import importlib
import os

_EXT = None
_TRIED = False
_MODULES = {"release": "_C", "debug": "_C_debug", "asan": "_C_asan"}


def variant() -> str:
    v = os.environ.get("JMAE_EXT", "release")
    if v not in _MODULES:
        raise ValueError(f"JMAE_EXT={v!r}: expected one of {sorted(_MODULES)}")
    return v


def load(required: bool | None = None):
    global _EXT, _TRIED
    if _EXT is not None:
        return _EXT
    if not _TRIED:
        _TRIED = True
        try:
            _EXT = importlib.import_module("jumbo_mae_tpu_amd." + _MODULES[variant()])
        except ImportError as e:  # pragma: no cover - depends on build state
            _EXT = None
            _err = e
            if required:
                raise RuntimeError(
                    "jumbo_mae_tpu_amd HIP extension not built: run "
                    "`python -m jumbo_mae_tpu_amd.csrc.build --variant " + variant() + "` (or "
                    "__graft_entry__.build())") from _err
    if _EXT is None and required:
        raise RuntimeError("jumbo_mae_tpu_amd HIP extension unavailable")
    return _EXT


def available() -> bool:
    return load(False) is not None


def use_hip(t) -> bool:
    """True when tensor ``t`` lives on the GPU and the fused kernels must be used."""
    if not t.is_cuda:
        return False
    if os.environ.get("JMAE_ALLOW_TORCH_FALLBACK", "0") == "1" and not available():
        return False
    load(True)
    return True


def debug_check() -> None:
    """Raise if a debug-build (``JMAE_EXT=debug``) device check has failed since the last call.
    No-op with the release extension (its ``debug_lines()`` is always empty)."""
    ext = load(False)
    if ext is None:
        return
    lines = ext.debug_lines()
    if lines:
        raise RuntimeError(f"HIP debug checks failed (translation unit -> csrc source line): {dict(lines)}")
