"""FF GELU epilogues: forward saving h (EPI_GELU) vs saving gelu'(h) (EPI_GELU_D), and the data
gradient through the GELU recomputing gelu'(h) (EPI_DGELU) vs multiplying by the saved derivative
(EPI_DMUL), at the ViT-L encoder / MAE-decoder FF shapes.  Interleaved rounds, one process.

    python tools/gelu_epi_bench.py [--iters 20 --rounds 3]
"""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.environ.get("JMAE_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jumbo_mae_tpu_amd.ops import _ext  # noqa: E402

# (M tokens, hidden N, width K)
SHAPES = {"enc": (25088, 4096, 1024), "dec": (101888, 2048, 512), "vitb": (25088, 3072, 768)}


def timeit(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--path", type=int, default=0, help="NT GEMM kernel path (ext.gemm_test_force), 0 = by shape")
    a = ap.parse_args()
    ext = _ext.load()
    ext.gemm_test_force(a.path)
    for name, (M, N, K) in SHAPES.items():
        x = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
        w1 = (torch.randn(N, K, device="cuda") * 0.03).bfloat16()
        b1 = torch.randn(N, device="cuda") * 0.1
        dy = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
        w2t = (torch.randn(N, K, device="cuda") * 0.03).bfloat16()  # W2^T [N, K]: dg = dy . W2
        pre, _ = ext.gemm_nt(x, w1, b1, True)
        gp, _ = ext.gemm_nt(x, w1, b1, True, False, True)
        db = torch.zeros(N, device="cuda")
        cases = {
            "fwd save h     ": lambda: ext.gemm_nt(x, w1, b1, True),
            "fwd save gelu' ": lambda: ext.gemm_nt(x, w1, b1, True, False, True),
            "dgrad gelu'(h) ": lambda: ext.gemm_nt_dgelu(dy, w2t, pre, db),
            "dgrad x saved  ": lambda: ext.gemm_nt_dgelu(dy, w2t, gp, db, True),
        }
        res = {k: [] for k in cases}
        for _ in range(a.rounds):
            for k, fn in cases.items():
                res[k].append(timeit(fn, a.iters))
        for k, v in res.items():
            us = min(v)
            print(f"{name} M={M} N={N} K={K} {k}: {us:8.1f} us  {2.0 * M * N * K / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
