"""AdamW multi-tensor kernel (csrc/optim.hip) alone on ViT-L-sized flat buffers (16 B per lane;
profiles/r3_adamw_streaming.txt: the pass runs at ~5.0 TB/s).

    python tools/adamw_bench.py [--n 400000000] [--rounds 5]"""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jumbo_mae_tpu_amd.ops import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=400_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--chunk", type=int, default=65536, help="elements per chunk-table row")
    a = ap.parse_args()
    ext = _ext.load()
    C = a.chunk
    n = a.n // C * C
    p, g = torch.randn(n, device="cuda") * 0.02, torch.randn(n, device="cuda") * 1e-3
    mu, nu = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    shadow = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    starts = torch.arange(0, n, C, dtype=torch.int32)
    chunks = torch.stack([starts, torch.full_like(starts, C), torch.zeros_like(starts)], 1).contiguous().cuda()
    meta = torch.tensor([1.0, 1.0, 0.0, 1.0], device="cuda")
    hyper = torch.tensor([1e-4, 0.1, 0.05, 1.0, 0.9, 0.95, 1e-8, 0.05], device="cuda")
    gn = torch.tensor([-1.0], device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(a.rounds):
        ext.opt_adamw(p, g, mu, nu, shadow, chunks, meta, hyper, gn)
        e0.record()
        for _ in range(a.iters):
            ext.opt_adamw(p, g, mu, nu, shadow, chunks, meta, hyper, gn)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / a.iters)
    tb = min(ts)
    print(f"adamw n={n} chunk={C}: {tb:8.1f} us (rounds {', '.join(f'{x:.0f}' for x in ts)})  "
          f"{30.0 * n / tb / 1e6:5.2f} TB/s at 30 B/param", flush=True)


if __name__ == "__main__":
    main()
