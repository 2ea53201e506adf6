"""TN MFMA weight-gradient GEMM (csrc/gemm_tn.hip) vs the hipBLASLt split-K path on the flagship
ViT-L Jumbo-MAE wgrad shapes (M tokens, N = Dense out, K = Dense in).  Interleaved timing."""

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jumbo_mae_tpu_amd.ops import _ext  # noqa: E402
from jumbo_mae_tpu_amd.ops.prims import wgrad_split  # noqa: E402

SHAPES = {
    "enc_qkv": (26624, 3072, 1024), "enc_wo": (26624, 1024, 1024), "enc_ff1": (25088, 4096, 1024),
    "enc_ff2": (25088, 1024, 4096), "jumbo1": (512, 12288, 3072), "jumbo2": (512, 3072, 12288),
    "dec_qkv": (101888, 1536, 512), "dec_wo": (101888, 512, 512), "dec_ff1": (101888, 2048, 512),
    "dec_ff2": (101888, 512, 2048), "patch": (25088, 1024, 768), "pred": (100352, 768, 512),
    # the headline's 2048-image micro-batch
    "enc_qkv_2k": (106496, 3072, 1024), "enc_wo_2k": (106496, 1024, 1024), "enc_ff1_2k": (100352, 4096, 1024),
    "enc_ff2_2k": (100352, 1024, 4096), "dec_qkv_2k": (407552, 1536, 512), "dec_wo_2k": (407552, 512, 512),
    "dec_ff1_2k": (407552, 2048, 512), "dec_ff2_2k": (407552, 512, 2048),
}


def blas(dy, x, g):
    M, N = dy.shape
    K = x.shape[1]
    s = wgrad_split(M, N, K)
    if s > 1:
        part = torch.bmm(dy.view(s, M // s, N).transpose(1, 2), x.view(s, M // s, K), out_dtype=torch.float32)
        _ext.load().splitk_reduce_add(part, g)
    else:
        torch.addmm(g, dy.t(), x, out_dtype=torch.float32, out=g)


def timeit(fn, iters=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    vs = [0]  # one TN kernel (the r1 / atomic / acc0 variants were removed; profiles/r1_*, r2_tn_*)
    ext = _ext.load()
    to_t = tb_t = 0.0
    for name, (M, N, K) in SHAPES.items():
        if a.only and name not in a.only.split(","):
            continue
        dy = (torch.rand(M, N, device="cuda") * 2 - 1).bfloat16()
        x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        g0 = torch.zeros(N, K, device="cuda")
        g1 = torch.zeros(N, K, device="cuda")
        S = ext.gemm_tn_wgrad(dy, x, g0)
        blas(dy, x, g1)
        err = ((g0 - g1).abs().max() / g1.abs().max()).item()
        tv = {v: [] for v in vs}
        tbs = []
        for _ in range(3):
            for v in vs:
                tv[v].append(timeit(lambda: ext.gemm_tn_wgrad(dy, x, g0)))
            tbs.append(timeit(lambda: blas(dy, x, g1)))
        to, tb = min(tv[vs[0]]), min(tbs)
        fl = 2.0 * M * N * K
        if len(vs) > 1:
            print("   " + "  ".join(f"v{v}: {min(tv[v]):7.1f} us {fl / min(tv[v]) / 1e6:5.0f} TF" for v in vs), flush=True)
        to_t += to
        tb_t += tb
        print(f"{name:8s} M={M:6d} N={N:5d} K={K:5d} S={S:3d}  ours {to:8.1f} us {fl / to / 1e6:6.0f} TF | "
              f"hipBLASLt split-K {tb:8.1f} us {fl / tb / 1e6:6.0f} TF | x{tb / to:4.2f}  relerr {err:.1e}", flush=True)
    print(f"total ours {to_t:.0f} us  hipBLASLt {tb_t:.0f} us")


if __name__ == "__main__":
    main()
