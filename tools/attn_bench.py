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

SHAPES = {"dec": (512, 199, 16, 32), "dec2k": (2048, 199, 16, 32), "enc": (512, 52, 16, 64), "enc2k": (2048, 52, 16, 64), "ft": (128, 199, 16, 64), "ft12": (128, 199, 12, 64)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default="dec,enc")
    a = ap.parse_args()
    ext = _ext.load()
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
            res = []
            for _ in range(3):
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res.append(e0.elapsed_time(e1) * 1e3 / a.iters)
            us = min(res)
            print(f"{name} {label} B={B} S={S} H={H} hd={hd}: {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
