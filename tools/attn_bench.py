"""Time the fused attention kernels at the flagship shapes (MAE decoder / Jumbo encoder).

    python tools/attn_bench.py [--iters N]

Prints one line per (shape, pass) with us/call and achieved TFLOP/s (useful flops only)."""

import argparse
import os
import sys

import torch

# JMAE_ROOT: package tree to import (A/B of two builds, tools/run_attn_ab.sh)
sys.path.insert(0, os.environ.get("JMAE_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from jumbo_mae_tpu_amd.ops import _ext  # noqa: E402

SHAPES = {"dec": (512, 199, 16, 32), "enc": (512, 52, 16, 64), "ft": (128, 199, 16, 64), "ft12": (128, 199, 12, 64)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default="dec,enc")
    ap.add_argument("--tr", type=int, default=-1, help="backward kernel (ext.attn_set_tr): 3 = batched bwd3 at hd 32, 2 = compact bwd2; -1 = default")
    ap.add_argument("--hpw", type=int, default=0, help="forward (b, h) pairs per workgroup, 0 = default")
    ap.add_argument("--ppw", type=int, default=0, help="backward batch elements per workgroup (bwd2), 0 = default")
    ap.add_argument("--remap", default="", help="comma list of attn_set_remap values to A/B (interleaved)")
    ap.add_argument("--max-seq", type=int, default=0, help="attn_set_max_seq (longer S -> tile-streamed kernels)")
    ap.add_argument("--bwd3-hd64", type=int, default=-1, help="attn_set_bwd3_hd64 (batched backward at hd 64)")
    ap.add_argument("--nw8", type=int, default=-1, help="attn_set_bwd3_nw8 (8-wave backward at hd 64, S > 64)")
    a = ap.parse_args()
    ext = _ext.load()
    remaps = [int(v) for v in a.remap.split(",")] if a.remap else [None]
    if a.ppw > 0:
        ext.attn_set_bwd_ppw(a.ppw)
    if a.hpw > 0:
        ext.attn_set_fwd_hpw(a.hpw)
    if a.tr >= 0:
        ext.attn_set_tr(a.tr)
    if a.max_seq > 0:
        ext.attn_set_max_seq(a.max_seq)
    if a.bwd3_hd64 >= 0:
        ext.attn_set_bwd3_hd64(a.bwd3_hd64)
    if a.nw8 >= 0:
        ext.attn_set_bwd3_nw8(a.nw8)
    for name in a.shapes.split(","):
        B, S, H, hd = SHAPES[name]
        D = H * hd
        qkv = (torch.randn(B, S, 3 * D, device="cuda") * 1.5).bfloat16()
        do = torch.randn(B, S, D, device="cuda").bfloat16()
        db = torch.zeros(3 * D, device="cuda") if S <= ext.attn_max_seq() else None
        o, lse = ext.attn_fwd(qkv, H)
        fl_f = 4.0 * B * H * S * S * hd
        for label, fn, fl in (("fwd", lambda: ext.attn_fwd(qkv, H), fl_f),
                              ("bwd", lambda: ext.attn_bwd(do, qkv, o, lse, H, db), 2.5 * fl_f)):
            res = {r: [] for r in remaps}
            for _ in range(3):
                for r in remaps:
                    if r is not None:
                        ext.attn_set_remap(r)
                    for _ in range(3):
                        fn()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    e0.record()
                    for _ in range(a.iters):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    res[r].append(e0.elapsed_time(e1) * 1e3 / a.iters)
            for r in remaps:
                us = min(res[r])
                tag = "" if r is None else f" remap={r}"
                print(f"{name} {label} B={B} S={S} H={H} hd={hd}{tag}: {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s",
                      flush=True)


if __name__ == "__main__":
    main()
