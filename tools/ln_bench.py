"""LayerNorm backward with the consumer's residual backward fused in (the production call of the
pretraining step: bf16 dy, fp32 residual input, residual-gradient add, branch-gradient output and
bias column sums) at the headline's 2048-image micro-batch shapes.

    python tools/ln_bench.py [--shapes dec2k,enc2k] [--iters 20]

Prints us per call and the achieved HBM rate over the bytes the pass must move (16 B / element;
14 B when x-hat is rebuilt from the bf16 LN output, ``--paths x,h``)."""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.environ.get("JMAE_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from jumbo_mae_tpu_amd.ops import _ext  # noqa: E402

SHAPES = {"dec2k": (2048, 199, 512), "enc2k": (2048, 52, 1024), "dec": (512, 199, 512), "enc": (512, 52, 1024)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="dec2k,enc2k")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--paths", default="x,h", help="x: read the fp32 input; h: rebuild x-hat from the bf16 output")
    a = ap.parse_args()
    ext = _ext.load()
    for name in a.shapes.split(","):
        B, T, D = SHAPES[name]
        x = torch.randn(B, T, D, device="cuda") * 2
        g, bt = torch.rand(D, device="cuda") + 0.5, torch.randn(D, device="cuda")
        h, mean, rstd = ext.layernorm_fwd(x, g, bt, 1e-6, torch.bfloat16)
        bt.clamp_(-0.5, 0.5)  # |beta| <= |gamma| everywhere: the h path applies (same h: timing only)
        dy = torch.randn(B * T, D, device="cuda").bfloat16()
        dres = torch.randn(B, T, D, device="cuda")
        y = torch.randn(B * T, D, device="cuda").bfloat16()
        z = lambda: torch.zeros(D, device="cuda")  # noqa: E731
        dg, db, dbi = z(), z(), z()
        for path in a.paths.split(","):
            hx = dict(hx=h, beta=bt) if path == "h" else {}
            fn = lambda: ext.layernorm_bwd(dy, x, mean, rstd, g, dg, db, True, dres, None, y, None, None,  # noqa: E731
                                           None, dbi, 0, None, **hx)
            res = []
            for _ in range(3):
                for _ in range(3):
                    fn()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                s.record()
                for _ in range(a.iters):
                    fn()
                e.record()
                torch.cuda.synchronize()
                res.append(s.elapsed_time(e) * 1e3 / a.iters)
            us = min(res)
            nb = 14 if path == "h" else 16
            print(f"{name} ln_bwd+residual ({path}) B={B} T={T} D={D}: {us:8.1f} us  {nb * B * T * D / us / 1e6:6.2f} TB/s",
                  flush=True)


if __name__ == "__main__":
    main()
