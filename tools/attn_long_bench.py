"""Long-sequence attention (S > 224, csrc/attention.hip tile-streamed kernels) vs the PyTorch
composition it replaced (fp32 einsum + logsumexp, hipBLAS batched GEMMs), forward and backward.

Shape: ViT-B/16 finetune at 448 px (S = 784 + 3 CLS = 787, 12 heads x 64), batch 32 per GPU.
  python tools/attn_long_bench.py [--batch 32] [--seq 787] [--heads 12] [--hd 64]
"""
import argparse
import math
import time

import torch

from jumbo_mae_tpu_amd.ops import _ext


def torch_fwd(qkv, H):
    B, S, D3 = qkv.shape
    hd = D3 // 3 // H
    q, k, v = qkv.float().view(B, S, 3, H, hd).unbind(2)
    z = torch.einsum("bqhd,bkhd->bhqk", q / math.sqrt(hd), k)
    lse = torch.logsumexp(z, -1)
    p = torch.exp(z - lse[..., None])
    return torch.einsum("bhqk,bkhd->bqhd", p, v).reshape(B, S, -1).to(qkv.dtype), lse


def torch_bwd(do, qkv, o, lse, H):
    B, S, D3 = qkv.shape
    hd = D3 // 3 // H
    q, k, v = qkv.float().view(B, S, 3, H, hd).unbind(2)
    dof = do.float().view(B, S, H, hd)
    sc = 1.0 / math.sqrt(hd)
    p = torch.exp(torch.einsum("bqhd,bkhd->bhqk", q * sc, k) - lse[..., None])
    dv = torch.einsum("bhqk,bqhd->bkhd", p, dof)
    dp = torch.einsum("bqhd,bkhd->bhqk", dof, v)
    delta = (dof * o.float().view(B, S, H, hd)).sum(-1).permute(0, 2, 1)
    ds = p * (dp - delta[..., None])
    dq = torch.einsum("bhqk,bkhd->bqhd", ds, k) * sc
    dk = torch.einsum("bhqk,bqhd->bkhd", ds, q) * sc
    return torch.stack([dq, dk, dv], 2).reshape(B, S, D3).to(qkv.dtype)


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=787)
    ap.add_argument("--heads", type=int, default=12)
    ap.add_argument("--hd", type=int, default=64)
    a = ap.parse_args()
    ext = _ext.load()
    B, S, H, hd = a.batch, a.seq, a.heads, a.hd
    torch.manual_seed(0)
    qkv = torch.randn(B, S, 3 * H * hd, device="cuda").bfloat16()
    do = torch.randn(B, S, H * hd, device="cuda").bfloat16()
    o, lse = ext.attn_fwd(qkv, H)
    flops_f = 4.0 * B * H * S * S * hd
    rows = []
    for name, f in (("hip fwd", lambda: ext.attn_fwd(qkv, H)),
                    ("hip bwd", lambda: ext.attn_bwd(do, qkv, o, lse, H)),
                    ("torch fwd", lambda: torch_fwd(qkv, H)),
                    ("torch bwd", lambda: torch_bwd(do, qkv, o, lse, H))):
        ms = f_ms = timeit(f)
        fl = flops_f * (2.5 if "bwd" in name else 1.0)
        rows.append(f"{name:10s} {ms:8.3f} ms  {fl / f_ms / 1e9:7.1f} TFLOP/s")
    print(f"# long-sequence attention B={B} S={S} H={H} hd={hd} (bf16 in/out, fp32 softmax)")
    print("\n".join(rows))


if __name__ == "__main__":
    main()
