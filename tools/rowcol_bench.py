"""Row/column kernels (csrc/elementwise.hip rowcol_kernel) at the small-M model shapes: the jumbo
residual backward (512 x 3072), the CLS-row attention residual backward (512 x 3 x 1024), the
jumbo GELU backward (512 x 12288) and a colsum.  python tools/rowcol_bench.py"""

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jumbo_mae_tpu_amd.ops import _ext  # noqa: E402


def timeit(fn, iters=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ext = _ext.load(True)
    for B, T, D in ((512, 1, 3072), (512, 3, 1024), (128, 1, 2304), (128, 3, 768)):
        dout = torch.randn(B, T, D, device="cuda")
        y = torch.randn(B * T, D, device="cuda").bfloat16()
        s = torch.rand(D, device="cuda")
        m = torch.rand(B, device="cuda")
        ds, db = torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
        t = timeit(lambda: ext.residual_bwd(dout, y, s, m, ds, torch.bfloat16, db))
        print(f"residual_bwd B={B} T={T} D={D}: {t:6.1f} us", flush=True)
    for M, N in ((512, 12288), (128, 9216)):
        h = torch.rand(M, N, device="cuda").bfloat16()
        da = torch.randn(M, N, device="cuda").bfloat16()
        bg = torch.zeros(N, device="cuda")
        t = timeit(lambda: ext.gelu_bwd(h, da, bg, True))
        print(f"gelu_bwd(deriv) M={M} N={N}: {t:6.1f} us", flush=True)
        t = timeit(lambda: ext.colsum(da, bg))
        print(f"colsum M={M} N={N}: {t:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
