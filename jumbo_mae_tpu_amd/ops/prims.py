"""Raw (non-autograd) primitives of the hot path with device dispatch.

GPU: fused CDNA4 HIP kernels (``jumbo_mae_tpu_amd._C``) + hipBLASLt GEMMs.  CPU: plain fp32
PyTorch that transcribes the reference math (the oracle).  Both the per-op autograd Functions
(ops/functional.py) and the fused transformer-block Functions (ops/blocks.py) are built from
these, so there is exactly one implementation of every op per device.

Parameter-gradient side effects: every ``*_bwd`` accumulates the gradients of the parameters it
owns into the flat fp32 gradient buffer and signals readiness to the data-parallel reducer.
"""

from __future__ import annotations

import contextlib
import math
import os

from typing import NamedTuple

import torch
import torch.nn.functional as F

from ..models.params import Handle
from . import _ext

LN_EPS = 1e-6
_GELU_C = math.sqrt(2.0 / math.pi)


def hip(t: torch.Tensor) -> bool:
    return _ext.use_hip(t)


def _trainable(h: Handle | None) -> bool:
    return h is not None and h.segs[0].trainable


# ------------------------------------------------------------------------------ GEMMs
def wgrad_split(M: int, N: int, K: int) -> int:
    """Split-K factor for a weight-gradient GEMM (reduction over M tokens, N x K output).

    A wgrad output is small (0.25-38 M elements) while its reduction is 25k-100k long, so one
    GEMM has only 4-200 256x256 output tiles for 256 CUs (measured 160-690 TF/s on MI355X,
    profiles/r1_gemm_wgrad_alternatives.log).  Splitting M into S chunks of one strided-batched
    GEMM gives S x tiles workgroups (fp32 partials, summed by one fused pass)."""
    tiles = max(1, (N // 256) * (K // 256))
    s = 1
    while s < 16 and tiles * s * 2 <= 256 and M % (s * 2) == 0 and M // (s * 2) >= 2048:
        s *= 2
    return s


_WGRAD_OURS = True


def wgrad(h: Handle, dy: torch.Tensor, x: torch.Tensor, rows: tuple[int, int] | None = None) -> None:
    """grad[h] += dy^T @ x  (fp32 accumulate; bf16 inputs on GPU); ``rows`` = (r0, r1) restricts
    it to gradient rows r0:r1 (``dy`` then holds only those output columns).

    GPU: the TN MFMA kernel (csrc/gemm_tn.hip, M split into fp32 partial tiles) for every shape
    with 256-aligned N, K and M >= 4096 -- 1.11-1.37x the hipBLASLt split-K path on the ViT-L
    Jumbo-MAE shapes (profiles/r1_wgrad_tn_vs_hipblaslt.txt); hipBLASLt otherwise."""
    g = h.grad if rows is None else h.grad[rows[0]:rows[1]]
    if dy.is_cuda and dy.dtype != torch.float32:
        M, N = dy.shape
        K = x.shape[1]
        if (_WGRAD_OURS and hip(dy) and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16
                and N % 256 == 0 and K % 256 == 0 and M >= 4096 and dy.stride(1) == 1 and x.stride(1) == 1):
            # whole-gradient writes may store (ParamStore.zero_grad skipped it); row slices settle
            store = h.take_store() if rows is None else False
            if rows is not None:
                h.settle()
            _ext.load().gemm_tn_wgrad(dy, x, g, store)
            return
        h.settle()  # the paths below accumulate
        if (_WGRAD_OURS and hip(dy) and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16
                and M < NARROW_MAX_M and K % 8 == 0):
            # short reduction (the classifier head, small batches): G^T-free NT form on the narrow
            # kernel, dW[N, K] = dy^T . x with the (zero-padded) token dim as the reduction
            g.add_(_ext.load().gemm_nt_f32(_pad_cols(dy.t()), _pad_cols(x.t())))
            return
        s = wgrad_split(M, N, K)
        if s > 1:
            part = torch.bmm(dy.view(s, M // s, N).transpose(1, 2), x.view(s, M // s, K), out_dtype=torch.float32)
            if hip(part):
                _ext.load().splitk_reduce_add(part, g)
            else:
                g.add_(part.sum(0))
        else:
            torch.addmm(g, dy.t(), x, out_dtype=torch.float32, out=g)
    else:
        g.addmm_(dy.t().float(), x.float())


def _tn_ok(dy: torch.Tensor, x: torch.Tensor) -> bool:
    """``wgrad`` runs this (dy, x) on the TN MFMA kernel (csrc/gemm_tn.hip)."""
    return (_WGRAD_OURS and hip(dy) and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and dy.dim() == 2
            and dy.shape[1] % 256 == 0 and x.shape[1] % 256 == 0 and dy.shape[0] >= 4096
            and dy.stride(1) == 1 and x.stride(1) == 1)


# ------------------------------------------------------------- paired weight gradients
# A weight gradient has only 16-64 256 x 256 output tiles (ViT-L: 1024 x 4096 -> 64), so the TN
# kernel splits the token reduction over S fp32 partial slices (S = 4-16) to fill 256 CUs, and a
# reduce pass sums them.  Inside a fused block's backward two consecutive weight gradients over the
# same token rows -- FF2 then FF1, Wo then QKV -- are held and launched as ONE grouped grid
# (gemm_tn_wgrad_group): twice the tiles, half the splits, half the partial bytes written and
# re-read.  The first one's ``ready`` waits for the pair.  A/B switch (module attribute): PAIR_WGRAD = False.
PAIR_WGRAD = True
_pair: dict = {"depth": 0, "held": None}


@contextlib.contextmanager
def paired_wgrads():
    _pair["depth"] += 1
    try:
        yield
    finally:
        _pair["depth"] -= 1
        if _pair["depth"] == 0:
            _flush_pair()


def _flush_pair() -> None:
    held, _pair["held"] = _pair["held"], None
    if held is not None:
        hw, dy, x = held
        wgrad(hw, dy, x)
        hw.ready()


def _wgrad_ready(hw: Handle, dy: torch.Tensor, x: torch.Tensor) -> None:
    """grad[hw] += dy^T x, then tell the reducer -- or hold it for / launch it with its pair."""
    if PAIR_WGRAD and _pair["depth"] > 0 and _tn_ok(dy, x):
        held = _pair["held"]
        if held is not None and held[1].shape[0] == dy.shape[0] and held[0] is not hw:
            _pair["held"] = None
            _ext.load().gemm_tn_wgrad_group([held[1], dy], [held[2], x], [held[0].grad, hw.grad],
                                            [held[0].take_store(), hw.take_store()])
            held[0].ready()
            hw.ready()
            return
        _flush_pair()
        _pair["held"] = (hw, dy, x)
        return
    wgrad(hw, dy, x)
    hw.ready()


def bias_grad(hb: Handle, dy: torch.Tensor) -> None:
    if hip(dy) and dy.dtype == torch.bfloat16 and dy.shape[-1] % 8 == 0 and dy.stride(-1) == 1:
        _ext.load().colsum(dy, hb.grad)
    else:
        hb.grad.add_(dy.sum(0, dtype=torch.float32))


_GEMM_MODE = "auto"  # auto | blas | ours (forward / dgrad routing)
_DGRAD_OURS = True  # data-gradient GEMMs on the MFMA kernel


NARROW_MAX_M = 4096  # csrc/gemm.hip NARROW_MAX_M: below it the NT GEMMs (split-K too) take 128 x 192 tiles
_NARROW_FUSED_MIN_TILES = 160  # a fused GELU epilogue needs the tiles alone to fill most CUs


def nt_tiles(M: int, N: int) -> int:
    """Output tiles of an NT launch on the tiles its M selects (the split-K / fused-epilogue
    decision below; jm_gemm_nt_tiles is exact: below NARROW_MAX_M the launch may take 4-phase
    tiles where they fill the chip's waves better, e.g. the N = 12288 jumbo GEMMs at M = 2048)."""
    if M < NARROW_MAX_M:
        return -(-M // 128) * -(-N // 192)
    return -(-M // 256) * -(-N // 256)


def use_our_gemm(M: int, N: int, K: int, fused_gelu: bool = False, kind: str = "fwd") -> bool:
    """Every forward / data-gradient Dense runs on a hand-written MFMA GEMM (csrc/gemm.hip): M >=
    4096 on the 256 x 256 4-phase kernel (it matches or beats hipBLASLt on the ViT-L step as a
    whole, profiles/r2_gemm_routing.txt), smaller M on the 128 x 192 narrow kernel (the 512-row
    jumbo MLP: one full wave of 256 tiles at N = 12288).  A fused GELU / dGELU epilogue is taken
    only when the narrow tiles alone fill most of the chip; otherwise the GEMM goes split-K
    (``splitk_plan``) and the GELU runs as its own kernel."""
    if _GEMM_MODE == "blas" or K % 64 or N % 8:
        return False
    if M >= NARROW_MAX_M:
        return True
    return not fused_gelu or nt_tiles(M, N) >= _NARROW_FUSED_MIN_TILES


def splitk_plan(M: int, N: int, K: int) -> int:
    """Split-K factor for a small-M GEMM whose narrow tiles cannot fill the chip (0 = not this path):
    the jumbo MLP's K = 12288 GEMMs (W2 forward, W1 data gradient: 24 256 x 256 tiles at M = 512 ->
    10 splits on the 4-phase kernel), the finetune jumbo MLP (M = 128: narrow tiles) and the
    classifier head.  Every split keeps >= 512 of K; fp32 partial slices are summed by one reduce
    (+ bias, or + an fp32 addend)."""
    if _GEMM_MODE == "blas" or M >= NARROW_MAX_M or K % 64 or N % 8:
        return 0
    if nt_tiles(M, N) >= _NARROW_FUSED_MIN_TILES:
        return 0
    s = min(256 // nt_tiles(M, N), K // 512, 16)
    return s if s >= 2 else 0


def _pad_cols(t: torch.Tensor, mult: int = 64) -> torch.Tensor:
    """[R, C] -> [R, ceil(C / mult) * mult] with zero columns (a reduction dim the MFMA kernels
    need in 64-deep steps, e.g. the 1000-class head's data gradient)."""
    c = t.shape[1]
    pad = -c % mult
    return F.pad(t, (0, pad)) if pad else t.contiguous()


def linear_fwd(x2: torch.Tensor, hw: Handle, hb: Handle | None) -> torch.Tensor:
    w = hw.weight()
    if hip(x2) and x2.dtype == torch.bfloat16:
        s = splitk_plan(x2.shape[0], w.shape[0], x2.shape[1])
        if s:
            return _ext.load().gemm_nt_splitk(x2, w, hb.master if hb is not None else None, s)
    if hip(x2) and x2.dtype == torch.bfloat16 and use_our_gemm(x2.shape[0], w.shape[0], x2.shape[1]):
        return _ext.load().gemm_nt(x2, w, hb.master if hb is not None else None, False)[0]
    if hb is not None:
        return torch.addmm(hb.weight(), x2, w.t())
    return x2 @ w.t()


def linear_gelu_fwd(x2: torch.Tensor, hw: Handle, hb: Handle | None, need_pre: bool = True):
    """(pre, gelu(pre)) of a Dense followed by the tanh GELU; one fused GEMM when it pays.
    ``need_pre=False`` (inference: no backward will read it) returns (None, gelu) and the fused
    epilogue writes only the activation."""
    w = hw.weight()
    if hip(x2) and x2.dtype == torch.bfloat16 and use_our_gemm(x2.shape[0], w.shape[0], x2.shape[1], True):
        if not need_pre:
            return None, _ext.load().gemm_nt(x2, w, hb.master if hb is not None else None, True, True)[0]
        pre, g = _ext.load().gemm_nt(x2, w, hb.master if hb is not None else None, True)
        return pre, g
    pre = linear_fwd(x2, hw, hb)
    return pre, gelu_fwd(pre)


# save gelu'(h) (8-bit codes) instead of h for the backward when the fused MFMA forward runs;
# JMAE_GELU_CODES=0: save h and recompute gelu'(h) exactly in the backward epilogue (loss-curve A/B
# of the two: profiles/r6b_gelu_code_loss_ab.txt)
_GELU_DERIV = os.environ.get("JMAE_GELU_CODES", "1") != "0"


# gelu'(h) saved as 8-bit codes by the fused FF1 forward (csrc/common.h gd_code): q = round(GD_Q d) + GD_Z
GD_Q, GD_Z = 195.0, 34


def gd_encode(d: torch.Tensor) -> torch.Tensor:
    """Torch mirror of the epilogue's gelu' code (tests): round to nearest even and saturate, as
    v_cvt_pk_u8_f32; the kernel's fma (one rounding) may differ by one code at exact ties."""
    return torch.clamp(torch.round(d.float() * GD_Q + GD_Z), 0, 255).to(torch.uint8)


def gd_decode(q: torch.Tensor, rate: float = 0.0, dtype=torch.bfloat16) -> torch.Tensor:
    """gelu'(h) from its codes; ``rate``: the forward's hidden dropout (codes of the unscaled kept value)."""
    s = (1.0 / (1.0 - rate) if rate > 0 else 1.0) / GD_Q
    return ((q.float() - GD_Z) * s).to(dtype)


def linear_gelu_fwd_saved(x2: torch.Tensor, hw: Handle, hb: Handle | None, need_pre: bool = True, drop=None):
    """Like ``linear_gelu_fwd`` but returns (saved, gelu(h), deriv, dropped): on the fused MFMA path
    the epilogue computes gelu(h) and gelu'(h) from one exp and ``saved`` is gelu'(h) as uint8 codes
    (deriv True, ``gd_decode``), so the backward's data-gradient epilogue multiplies instead of
    re-deriving it from h and reads 1 byte per element; otherwise ``saved`` is h (deriv False).
    ``drop`` = (seed, rate): hidden dropout applied inside that epilogue (dropped True; the codes
    hold the unscaled kept derivative, 1 / keep is applied when the backward decodes them); the
    other paths leave it to the caller."""
    w = hw.weight()
    if (_GELU_DERIV and need_pre and hip(x2) and x2.dtype == torch.bfloat16 and w.shape[0] % 8 == 0
            and use_our_gemm(x2.shape[0], w.shape[0], x2.shape[1], True)):
        bias = hb.master if hb is not None else None
        if drop is not None:
            gp, g = _ext.load().gemm_nt(x2, w, bias, True, False, True, drop[0], drop[1])
            return gp, g, True, True
        gp, g = _ext.load().gemm_nt(x2, w, bias, True, False, True)
        return gp, g, True, False
    pre, g = linear_gelu_fwd(x2, hw, hb, need_pre)
    return pre, g, False, False


# ------------------------------------------------------------------ weight-gradient stream
# The weight-gradient GEMMs are off the backward critical path (nothing in the backward reads
# them), so they run on a second HIP stream: hipBLASLt's 4-wave, <=256-VGPR workgroups leave
# room on every CU for the memory-bound LayerNorm / GELU / residual / attention kernels of the
# data-gradient chain, which then execute underneath them instead of after them.  The chain's
# tensors are pinned for the side stream with record_stream; the DP reducer launches its
# all-reduces from this stream and the trainer joins it before the optimizer.
# Off by default.  Round 1 (hipBLASLt wgrads): +1-2 % on most runs, some runs collapsed to
# 0.4-0.6x.  Round 2 (TN MFMA wgrads): no collapse in 6 processes, +0.3-0.8 %, and ~0.5 ms/step of
# cross-queue hand-off gaps in the trace (profiles/r2_wgrad_side_stream.txt); kept off so the DP
# reducer's collectives stay on the compute stream in multi-GPU runs.
_side = {"stream": None, "enabled": False, "cb": False}


def _end_of_backward() -> None:
    _side["cb"] = False
    join_wgrad_stream()


# ------------------------------------------------------------- deferred (batched) wgrad
# A weight used by every layer -- the shared jumbo MLP -- gets 24 weight-gradient GEMMs of only
# 512 rows (one per layer, ~400 TF/s on hipBLASLt).  Their (dy, x) pairs are queued and, at the
# end of the backward pass, concatenated into ONE GEMM over 24 x 512 rows on the TN MFMA kernel.
# The DP reducer is told the segment is ready only then (one ``ready`` per queued use).
_deferred: dict = {"handles": [], "cb": False, "enabled": True,
                   "force": False,  # also on CPU / fp32 (tests of the deferred + partial-reduce path)
                   "chunks": 4,
                   "seg": True}  # in-place segmented GEMM


def _row_chunks(n: int, want: int, align: int = 256) -> list[tuple[int, int]]:
    """Split n gradient rows into <= ``want`` chunks whose sizes are multiples of ``align`` (256 =
    the TN kernel's tile) when possible."""
    for c in range(want, 1, -1):
        if n % c == 0 and (n // c) % align == 0:
            step = n // c
            return [(i * step, (i + 1) * step) for i in range(c)]
    return [(0, n)]


def _seg_ok(dys, xs) -> bool:
    """The per-layer (dy, x) blocks can feed the segmented TN kernel in place (no concat)."""
    d0, x0 = dys[0], xs[0]
    return (_WGRAD_OURS and _deferred["seg"] and hip(d0) and len(dys) <= 32 and d0.shape[0] % 32 == 0
            and d0.shape[1] % 256 == 0 and x0.shape[1] % 256 == 0
            and all(d.dtype == torch.bfloat16 and d.shape == d0.shape and d.stride() == d0.stride() for d in dys)
            and all(x.dtype == torch.bfloat16 and x.shape == x0.shape and x.stride() == x0.stride() for x in xs)
            and d0.stride(1) == 1 and x0.stride(1) == 1)


GROUP_JUMBO_WGRAD = True  # A/B switch


def _flush_seg_group(todo: list) -> list:
    """Batched weight gradients of two shared weights over the same per-layer row blocks (the
    jumbo MLP's W1 and W2) as ONE grouped segmented grid, when neither needs chunked partial
    readiness for the DP reducer: twice the tiles, so no M split and no partial slices to reduce
    (gemm_tn_wgrad_seg_group).  Returns the entries left for the per-handle path."""
    if not GROUP_JUMBO_WGRAD or len(todo) != 2:
        return todo
    (h1, p1), (h2, p2) = todo
    if any(h.store.partial_hooks and len(h.segs) == 1 for h in (h1, h2)) or len(p1) != len(p2):
        return todo
    d1, x1 = [p[0] for p in p1], [p[1] for p in p1]
    d2, x2 = [p[0] for p in p2], [p[1] for p in p2]
    if not (_seg_ok(d1, x1) and _seg_ok(d2, x2) and d1[0].shape[0] == d2[0].shape[0]
            and d1[0].shape[0] % 64 == 0 and h1.grad.is_contiguous() and h2.grad.is_contiguous()):
        return todo
    _ext.load().gemm_tn_wgrad_seg_group([d1, d2], [x1, x2], [h1.grad, h2.grad], [h1.take_store(), h2.take_store()])
    for h, pairs in todo:
        for _ in pairs:
            h.ready()
    return []


def flush_deferred_wgrads() -> None:
    _deferred["cb"] = False
    hs, _deferred["handles"] = _deferred["handles"], []
    todo = []
    for h in hs:
        pairs, h.deferred = h.deferred, []
        if pairs:
            todo.append((h, pairs))
    for h, pairs in _flush_seg_group(todo):
        dys = [p[0] for p in pairs]
        xs = [p[1] for p in pairs]
        N, K = dys[0].shape[1], xs[0].shape[1]
        chunks = [(0, N)]
        if h.store.partial_hooks and len(h.segs) == 1:
            chunks = _row_chunks(N, _deferred["chunks"], 256 if hip(dys[0]) else 32)
        seg = _seg_ok(dys, xs)
        if not seg:
            dy = torch.cat(dys) if len(dys) > 1 else dys[0]
            x = torch.cat(xs) if len(xs) > 1 else xs[0]
        store = h.take_store() if seg else False  # every chunk is its rows' only contribution
        if len(chunks) > 1 and not seg:
            h.settle()
        for r0, r1 in chunks:
            if seg:  # the batched GEMM reads the 24 per-layer blocks in place
                _ext.load().gemm_tn_wgrad_seg([d[:, r0:r1] for d in dys], xs, h.grad[r0:r1], store)
            elif len(chunks) == 1:
                wgrad(h, dy, x)
            else:
                wgrad(h, dy[:, r0:r1], x, rows=(r0, r1))
            if len(chunks) > 1:  # these gradient rows are final: the DP reducer starts on them at once
                h.store.mark_partial_ready(h, r0 * K, r1 * K)
        for _ in pairs:
            h.ready()


def _defer_wgrad(hw: Handle, dy: torch.Tensor, x2: torch.Tensor) -> bool:
    """Queue (dy, x) for the batched GEMM; False when not inside an autograd backward pass."""
    if not _deferred["cb"]:
        try:
            torch.autograd.Variable._execution_engine.queue_callback(flush_deferred_wgrads)
        except RuntimeError:
            return False
        _deferred["cb"] = True
    if not hw.deferred:
        _deferred["handles"].append(hw)
    hw.deferred.append((dy, x2))
    return True


def wgrad_stream():
    """The side stream (created lazily), or None when disabled / not on a GPU."""
    if not _side["enabled"] or not torch.cuda.is_available():
        return None
    if _side["stream"] is None:
        _side["stream"] = torch.cuda.Stream()
    return _side["stream"]


def set_wgrad_stream(enabled: bool) -> None:
    _side["enabled"] = bool(enabled)


def join_wgrad_stream() -> None:
    """Make the current stream wait for every queued weight-gradient GEMM."""
    s = _side["stream"]
    if s is not None:
        torch.cuda.current_stream().wait_stream(s)


def linear_dgrad(dy: torch.Tensor, hw: Handle, add: torch.Tensor | None = None) -> torch.Tensor:
    """dx = dy @ W: on the MFMA kernel against the transposed weight copy when it wins.  With
    ``add`` (fp32 [M, N]) the fp32 sum ``add + dy @ W`` is returned (fused into the split-K
    reduction on the jumbo-MLP path)."""
    w = hw.weight()
    if _DGRAD_OURS and hip(dy) and dy.dtype == torch.bfloat16:
        s = splitk_plan(dy.shape[0], w.shape[1], w.shape[0])
        if (not s and add is not None and dy.shape[0] < NARROW_MAX_M and w.shape[0] % 64 == 0
                and w.shape[1] % 8 == 0 and _GEMM_MODE != "blas"):
            # fp32 addend below the narrow-tile bound (the jumbo W1 data gradient at a 2048-row
            # micro-batch): one fp32 "split" and the reduce's add instead of a bf16 output, an
            # upcast copy and a torch add (same narrow kernel, 3 -> 2 launches, 125 -> 100 MB)
            s = 1
        if s:
            if add is not None and add.stride(-1) == 1 and add.stride(0) % 4 == 0 and add.shape[1] % 4 == 0:
                return _ext.load().gemm_nt_splitk(dy.contiguous(), hw.weight_t(), None, s, add)
            dx = _ext.load().gemm_nt_splitk(dy.contiguous(), hw.weight_t(), None, s)
            return dx if add is None else add + dx.float()
    if add is not None:
        return add + linear_dgrad(dy, hw).float()
    if (_DGRAD_OURS and hip(dy) and dy.dtype == torch.bfloat16
            and use_our_gemm(dy.shape[0], w.shape[1], w.shape[0], kind="dgrad")):
        return _ext.load().gemm_nt(dy.contiguous(), hw.weight_t(), None, False)[0]
    if (_DGRAD_OURS and hip(dy) and dy.dtype == torch.bfloat16 and w.shape[0] % 64
            and use_our_gemm(dy.shape[0], w.shape[1], -(-w.shape[0] // 64) * 64, kind="dgrad")):
        # reduction dim (the Dense's output width, e.g. 1000 classes) zero-padded to 64-deep steps
        return _ext.load().gemm_nt(_pad_cols(dy), _pad_cols(hw.weight_t()), None, False)[0]
    return dy @ w


def linear_bwd(dy: torch.Tensor, x2: torch.Tensor, hw: Handle, hb: Handle | None, need_dx: bool = True,
               bias_done: bool = False, dx_add: torch.Tensor | None = None):
    """dx = dy @ W (if needed; ``dx_add + dy @ W`` in fp32 with ``dx_add``); grad W += dy^T x;
    grad b += colsum(dy) (unless fused upstream)."""
    dx = linear_dgrad(dy, hw, dx_add) if need_dx else None
    if (_trainable(hw) and hw.defer_wgrad and _deferred["enabled"] and (hip(dy) or _deferred["force"])
            and _defer_wgrad(hw, dy, x2)):
        if hb is not None:
            if not bias_done:
                bias_grad(hb, dy)
            hb.ready()
        return dx
    if _trainable(hw):
        side = wgrad_stream() if dy.is_cuda else None
        if side is not None:
            if not _side["cb"]:  # the backward pass returns only after joining the side stream
                torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)
                _side["cb"] = True
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                wgrad(hw, dy, x2)
                if hb is not None and not bias_done:
                    bias_grad(hb, dy)
            dy.record_stream(side)
            x2.record_stream(side)
            hw.ready()
        else:
            if hb is not None and not bias_done:
                bias_grad(hb, dy)
            _wgrad_ready(hw, dy, x2)
        if hb is not None:
            hb.ready()
    return dx


def linear_gelu_bwd(dy: torch.Tensor, g: torch.Tensor, pre: torch.Tensor, hw2: Handle, hb2: Handle | None,
                    hb1: Handle | None, bias2_done: bool = False, deriv: bool = False, rate: float = 0.0):
    """Backward of ``y = Dense2(gelu(pre))`` down to d pre: returns (dpre, bias1_done).

    Fused path: one MFMA GEMM dy . W2 whose epilogue multiplies by gelu'(pre) and emits the
    column sums of dpre (= the gradient of Dense1's bias ``hb1``), so the GEMM output dg never
    makes an HBM round trip.  W2's own gradients (wgrad, bias) are queued as usual.  ``deriv``:
    ``pre`` is the saved gelu'(h) (``linear_gelu_fwd_saved``; uint8 codes), not h; ``rate``: the
    forward's hidden dropout rate folded into those codes."""
    w2 = hw2.weight()
    M, N, K = dy.shape[0], w2.shape[1], w2.shape[0]
    if (_DGRAD_OURS and hip(dy) and dy.dtype == torch.bfloat16 and N % 8 == 0
            and (not deriv or pre.dtype == torch.uint8)  # a bf16 gelu' (unfused forward) takes gelu_bwd
            and use_our_gemm(M, N, K, fused_gelu=True, kind="dgrad")):
        bg = hb1.grad if _trainable(hb1) else None
        dpre = _ext.load().gemm_nt_dgelu(dy.contiguous(), hw2.weight_t(), pre.contiguous(), bg, deriv, rate)
        linear_bwd(dy, g, hw2, hb2, need_dx=False, bias_done=bias2_done)
        return dpre, bg is not None
    if deriv and pre.dtype == torch.uint8:
        pre = gd_decode(pre, rate, dy.dtype)
    dg = linear_bwd(dy, g, hw2, hb2, bias_done=bias2_done)
    return gelu_bwd(pre, dg, hb1, deriv)


# ------------------------------------------------------------------------------ gelu
def gelu_fwd(h: torch.Tensor) -> torch.Tensor:
    if hip(h):
        return _ext.load().gelu_fwd(h)
    return F.gelu(h, approximate="tanh")


def gelu_bwd(h: torch.Tensor, da: torch.Tensor, hb: Handle | None = None,
             deriv: bool = False) -> tuple[torch.Tensor, bool]:
    """dh = da * gelu'(h) (``deriv``: h already holds gelu'); when ``hb`` is given its bias gradient
    (colsum dh) is fused in.  Returns (dh, bias_done)."""
    if hip(h):
        bg = hb.grad if _trainable(hb) else None
        return _ext.load().gelu_bwd(h, da.contiguous(), bg, deriv), bg is not None
    if deriv:
        return (da.float() * h.float()).to(h.dtype), False
    hf = h.float()
    u = _GELU_C * (hf + 0.044715 * hf ** 3)
    t = torch.tanh(u)
    d = 0.5 * (1 + t) + 0.5 * hf * (1 - t * t) * _GELU_C * (1 + 3 * 0.044715 * hf * hf)
    return (da.float() * d).to(h.dtype), False


# ------------------------------------------------------------------------------ layernorm
def ln_fwd(x3: torch.Tensor, hg: Handle, hb: Handle, out_dtype, also_dtype=None):
    """x3: fp32 [B, T, D] view -> (y [B*T, D], mean, rstd); with ``also_dtype`` (fp32 ``y`` only) a
    copy of y in that dtype is returned 4th, written by the same pass on the GPU."""
    B, T, D = x3.shape
    if hip(x3):
        if also_dtype is not None and out_dtype == torch.float32 and also_dtype == torch.bfloat16:
            return tuple(_ext.load().layernorm_fwd(x3, hg.master, hb.master, LN_EPS, out_dtype, True))
        out = tuple(_ext.load().layernorm_fwd(x3, hg.master, hb.master, LN_EPS, out_dtype))
        return out if also_dtype is None else out + (out[0].to(also_dtype),)
    xf = x3.reshape(B * T, D).float()
    mean = xf.mean(-1)
    var = (xf - mean[:, None]).square().mean(-1)
    rstd = torch.rsqrt(var + LN_EPS)
    y = ((xf - mean[:, None]) * rstd[:, None] * hg.master + hb.master).to(out_dtype)
    return (y, mean, rstd) if also_dtype is None else (y, mean, rstd, y.to(also_dtype))


_FUSE_LN_RES = True  # A/B switch (tools/ab_bench.py)


class ResSpec(NamedTuple):
    """Residual backward that consumes a LayerNorm backward's dx (fused into it by ``ln_bwd``):
    for rows t >= t0, dy = mask[b] * s * dx in bf16; s.grad += colsum(mask * dx * y);
    hbias.grad += colsum(dy).  ``y`` is the branch output of those rows ([B*(T-t0), D] contiguous
    or a [B, T-t0, D] view); ``out`` an optional destination view with y's layout; ``drop`` the
    branch output's dropout (see ``_drop_args``)."""
    y: torch.Tensor
    hs: Handle | None
    mask: torch.Tensor | None
    hbias: Handle | None
    t0: int = 0
    out: torch.Tensor | None = None
    drop: tuple | None = None


def _drop_args(y: torch.Tensor, drop) -> tuple:
    """Kernel arguments (seed, rate, ioff) of the Dense-output dropout ``drop`` = (seed, rate, base):
    the mask indexes the branch tensor ``base`` (flat), ``y`` is a view of it."""
    if drop is None:
        return None, 0.0, 0
    seed, rate, base = drop
    return seed, rate, y.storage_offset() - base.storage_offset()


def _drop_factor(y: torch.Tensor, drop) -> torch.Tensor:
    """fp32 keep / keep_p factors in ``y``'s layout (CPU path of the residual kernels' dropout)."""
    from . import dropout as Dr
    seed, rate, base = drop
    _, scale = Dr.keep_threshold(rate)
    full = Dr.keep_mask(seed.cpu(), base.numel(), rate).to(y.device).float() * scale
    return full.as_strided(y.shape, y.stride(), y.storage_offset() - base.storage_offset())


# LN backward rebuilding x-hat from the forward's bf16 output h = bf16(gamma x-hat + beta) when every
# column has |beta| <= |gamma| (2 bytes per element instead of the fp32 input's 4; csrc/layernorm.hip
# LnBwdIO).  OFF: measured 8-9 % slower per LN backward and 0.4 % per step despite the 12.5 % fewer
# bytes -- the pass is bound by its per-row latency chain, not HBM bytes
# (profiles/r6d_ln_bwd_from_h.txt); kept as a tested switch (ab_bench LN_FROM_H=1).
_LN_BWD_FROM_H = False


def ln_bwd(dy: torch.Tensor, x3: torch.Tensor, mean, rstd, hg: Handle, hb: Handle, dres=None, out=None,
           res: ResSpec | None = None, h: torch.Tensor | None = None):
    """dx = LN'(dy) (+ dres) written to ``out`` (a [B,T,D] view) or a new tensor; accumulates
    dgamma / dbeta.  With ``res`` the residual backward of dx's consumer rides on the same pass
    and (dx, dy_res, bias_done) is returned (the separate pass would re-read dx from HBM).
    ``h``: the forward's bf16 output of this LN (rows like ``dy``); the HIP kernel then reads it
    instead of ``x3`` when every column has |beta| <= |gamma| (x-hat exact to bf16 level)."""
    B, T, D = x3.shape
    dy = dy.contiguous()
    tr = _trainable(hg)
    fused = res is not None and _FUSE_LN_RES and hip(x3) and res.y.dtype == torch.bfloat16
    dyr = None
    if hip(x3):
        hx = h if (_LN_BWD_FROM_H and h is not None and h.dtype == torch.bfloat16 and h.is_contiguous()
                   and h.numel() == dy.numel()) else None
        beta = hb.master if hx is not None else None
        if fused:
            hs, hbias = res.hs, res.hbias
            dseed, drate, dioff = _drop_args(res.y, res.drop)
            dx, dyr = _ext.load().layernorm_bwd(
                dy, x3, mean, rstd, hg.master, hg.grad, hb.grad, tr, dres, out, res.y,
                hs.master if hs is not None else None, res.mask, hs.grad if _trainable(hs) else None,
                hbias.grad if _trainable(hbias) else None, res.t0, res.out, dseed, drate, dioff, hx, beta)
        else:
            dx = _ext.load().layernorm_bwd(dy, x3, mean, rstd, hg.master, hg.grad, hb.grad, tr, dres, out,
                                           hx=hx, beta=beta)[0]
    else:
        xf = x3.reshape(B * T, D).float()
        xhat = (xf - mean[:, None]) * rstd[:, None]
        dyf = dy.reshape(B * T, D).float()
        if tr:
            hg.grad.add_((dyf * xhat).sum(0))
            hb.grad.add_(dyf.sum(0))
        g = dyf * hg.master
        dx = rstd[:, None] * (g - g.mean(-1, keepdim=True) - xhat * (g * xhat).mean(-1, keepdim=True))
        dx = dx.reshape(B, T, D)
        if dres is not None:
            dx = dx + dres
        if out is not None:
            out.copy_(dx)
            dx = out
    if tr:
        hg.ready()
        hb.ready()
    if res is None:
        return dx
    if fused:
        if _trainable(res.hs):
            res.hs.ready()
        return dx, dyr, _trainable(res.hbias)
    dyr, done = residual_bwd(dx[:, res.t0:], res.y, res.hs, res.mask, res.y.dtype, res.hbias, out=res.out,
                             drop=res.drop)
    return dx, dyr, done


# ------------------------------------------------------------------------------ residual
def residual_fwd(x3: torch.Tensor, y2: torch.Tensor, hs: Handle | None, mask, out=None, drop=None) -> torch.Tensor:
    """out[b,t] = x[b,t] + mask[b] * s * y[b*T+t]  (x, out: fp32 [B,T,D] views); ``drop``: the
    dropout of y (seed, rate, base tensor), applied as y is read."""
    B, T, D = x3.shape
    if hip(x3):
        y2r = y2.reshape(B * T, D)
        dseed, drate, dioff = _drop_args(y2r, drop)
        return _ext.load().residual_fwd(x3, y2r, hs.master if hs is not None else None, mask, out, dseed, drate,
                                        dioff)
    r = y2.float()
    if drop is not None:
        r = r * _drop_factor(y2, drop)
    r = r.reshape(B, T, D)
    if hs is not None:
        r = r * hs.master
    if mask is not None:
        r = r * mask.view(B, 1, 1)
    res = x3.float() + r
    if out is not None:
        out.copy_(res)
        return out
    return res


def residual_ln_fwd(x3: torch.Tensor, y2: torch.Tensor, hs: Handle | None, mask, hg: Handle, hb: Handle,
                    t0: int = 0, r0: int = 0, out: torch.Tensor | None = None, drop=None):
    """x1 = x + mask*s*y (fresh [B,T,D] fp32, or ``out``) and the LayerNorm of its rows t >= t0 in
    one pass: returns (x1, h [B*(T-t0), D] bf16, mean, rstd).  The fused kernel saves the LN's re-read
    of x1.  ``r0 > 0``: only rows t >= r0 get the residual (``y2`` holds those rows); rows t < r0
    of ``out`` are already final and are only normalised."""
    B, T, D = x3.shape
    if hip(x3) and y2.dtype == torch.bfloat16:
        if drop is not None:  # the kernel indexes y's own rows: y must be its branch tensor
            assert y2.data_ptr() == drop[2].data_ptr() and y2.numel() == drop[2].numel()
        return tuple(_ext.load().residual_ln_fwd(x3, y2.reshape(B * (T - r0), D),
                                                 hs.master if hs is not None else None, mask, hg.master, hb.master,
                                                 LN_EPS, t0, r0, out, drop[0] if drop else None,
                                                 drop[1] if drop else 0.0))
    if r0 == 0 and out is None:
        x1 = residual_fwd(x3, y2, hs, mask, drop=drop)
    else:
        x1 = out if out is not None else torch.empty_like(x3)
        residual_fwd(x3[:, r0:], y2, hs, mask, out=x1[:, r0:], drop=drop)
    h, mean, rstd = ln_fwd(x1[:, t0:], hg, hb, hg.store.compute_dtype)
    return x1, h, mean, rstd


def residual_bwd(dout3: torch.Tensor, y2: torch.Tensor | None, hs: Handle | None, mask, ydtype,
                 hbias: Handle | None = None, out: torch.Tensor | None = None, mark_ready: bool = True, drop=None):
    """dy = mask[b] * s * dout (in ``ydtype``); ds += sum mask*dout*y.  When ``hbias`` (the bias of
    the Dense that produced y) is given, its gradient colsum(dy) is fused into the same pass.
    ``y2``: [B*T, D] or a [B, T, D] view; ``out``: optional destination view with y2's layout.
    ``mark_ready=False`` leaves s's reducer readiness to a later contributor.  Returns (dy, bias_done)."""
    B, T, D = dout3.shape
    bg = hbias.grad if _trainable(hbias) else None
    if hip(dout3) and ydtype == torch.bfloat16 and (hs is not None or mask is not None or bg is not None
                                                    or drop is not None):
        dseed, drate, dioff = _drop_args(y2 if y2 is not None else out, drop)
        dy = _ext.load().residual_bwd(dout3, y2, hs.master if hs is not None else None, mask,
                                      hs.grad if _trainable(hs) else None, ydtype, bg, out, dseed, drate, dioff)
        done = bg is not None
    else:
        d = dout3.float()
        if mask is not None:
            d = d * mask.view(B, 1, 1)
        if drop is not None:  # d(y_pre) = keep * d(y_dropped); the scale gradient sees the dropped y
            d = d * _drop_factor(y2, drop).reshape(B, T, D)
        if hs is not None:
            if _trainable(hs):
                hs.grad.add_((d * y2.float().reshape(B, T, D)).sum((0, 1)))
            d = d * hs.master
        dy = d.to(ydtype)
        if out is not None:
            out.copy_(dy.reshape(out.shape))
            dy = out
        else:
            dy = dy.reshape(B * T, D)
        done = False
    if mark_ready and _trainable(hs):
        hs.ready()
    return dy, done


# ------------------------------------------------------------------------------ attention
def _attn_hip(qkv: torch.Tensor, heads: int) -> bool:
    """HIP attention covers head dims 32 / 64 at any length: the fused whole-sequence-in-LDS
    kernels up to S = attn_max_seq() (224: every flagship shape), tile-streamed online-softmax
    kernels beyond (e.g. finetuning at 448 px, S = 787).  Other head dims take
    the PyTorch composition below (fp32 softmax, same numerics)."""
    if not hip(qkv):
        return False
    hd = qkv.shape[2] // 3 // heads
    return hd in (32, 64)


def _drop_mask(drop, B: int, heads: int, S: int, device):
    """float [B, H, S, S] keep mask / keep of attention-probability dropout ``drop`` = (seed, rate):
    the fused kernels' index convention (ops/dropout.py keep_mask_rows), for the composition path."""
    from . import dropout as Dr
    seed, rate = drop
    _, scale = Dr.keep_threshold(rate)
    m = Dr.keep_mask_rows(seed.cpu(), B * heads * S, S, rate).view(B, heads, S, S).to(device)
    return m.float() * scale


def attn_fwd(qkv: torch.Tensor, heads: int, drop=None):
    """qkv [B, S, 3*D] -> (o [B, S, D], lse [B, H, S]).  ``drop`` = (seed int64 [1] tensor, rate):
    dropout on the attention probabilities (reference modeling.py:137), fused into the kernels up
    to S = attn_max_seq(); lse is that of the undropped softmax."""
    B, S, three_d = qkv.shape
    D = three_d // 3
    hd = D // heads
    if _attn_hip(qkv, heads) and (drop is None or S <= _ext.load().attn_max_seq()):
        if drop is None:
            return _ext.load().attn_fwd(qkv, heads)
        return _ext.load().attn_fwd(qkv, heads, drop[0], drop[1])
    q, k, v = qkv.float().view(B, S, 3, heads, hd).unbind(2)
    z = torch.einsum("bqhd,bkhd->bhqk", q / math.sqrt(hd), k)
    lse = torch.logsumexp(z, -1)
    p = torch.exp(z - lse[..., None])
    if drop is not None:
        p = p * _drop_mask(drop, B, heads, S, qkv.device)
    o = torch.einsum("bhqk,bkhd->bqhd", p, v).reshape(B, S, D).to(qkv.dtype)
    return o, lse


def attn_bwd(do: torch.Tensor, qkv: torch.Tensor, o: torch.Tensor, lse: torch.Tensor, heads: int,
             hbias: Handle | None = None, drop=None):
    """-> (dqkv [B, S, 3D], bias_done).  When ``hbias`` (the QKV Dense bias) is given, its gradient
    colsum(dqkv) is fused into the HIP kernel.  ``drop``: the forward's (seed, rate)."""
    B, S, three_d = qkv.shape
    D = three_d // 3
    hd = D // heads
    do = do.contiguous().view(B, S, D)
    if _attn_hip(qkv, heads) and (drop is None or S <= _ext.load().attn_max_seq()):
        ext = _ext.load()
        bg = hbias.grad if _trainable(hbias) and S <= ext.attn_max_seq() else None
        if drop is None:
            return ext.attn_bwd(do, qkv, o, lse, heads, bg), bg is not None
        return ext.attn_bwd(do, qkv, o, lse, heads, bg, drop[0], drop[1]), bg is not None
    q, k, v = qkv.float().view(B, S, 3, heads, hd).unbind(2)
    dof = do.float().view(B, S, heads, hd)
    sc = 1.0 / math.sqrt(hd)
    z = torch.einsum("bqhd,bkhd->bhqk", q * sc, k)
    p = torch.exp(z - lse[..., None])
    mk = _drop_mask(drop, B, heads, S, qkv.device) if drop is not None else None
    dv = torch.einsum("bhqk,bqhd->bkhd", p if mk is None else p * mk, dof)
    dp = torch.einsum("bqhd,bkhd->bhqk", dof, v)
    if mk is not None:
        dp = dp * mk
    delta = (dof * o.float().view(B, S, heads, hd)).sum(-1).permute(0, 2, 1)
    ds = p * (dp - delta[..., None])
    dq = torch.einsum("bhqk,bkhd->bqhd", ds, k) * sc
    dk = torch.einsum("bhqk,bqhd->bkhd", ds, q) * sc
    return torch.stack([dq, dk, dv], 2).reshape(B, S, three_d).to(qkv.dtype), False
