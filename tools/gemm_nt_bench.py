"""Our MFMA GEMM (ext.gemm_nt) vs hipBLASLt (torch) on the flagship ViT-L Jumbo-MAE shapes.

    python tools/gemm_nt_bench.py [--iters N] [--only name,...]

fwd shapes: x[M,K] @ W[N,K]^T + b.  dgrad shapes: dy[M,N] @ W[N,K] given to our kernel as
NT against the transposed weight W^T[K,N].  Interleaved timing in one process (A/B rounds)."""

import argparse
import os
import re
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jumbo_mae_tpu_amd.ops import _ext  # noqa: E402
from jumbo_mae_tpu_amd.ops import prims as P  # noqa: E402

FWD = {
    "enc_qkv": (26624, 3072, 1024), "enc_wo": (26624, 1024, 1024), "enc_ff1": (25088, 4096, 1024),
    "enc_ff2": (25088, 1024, 4096), "jumbo1": (512, 12288, 3072), "jumbo2": (512, 3072, 12288),
    "dec_qkv": (101888, 1536, 512), "dec_wo": (101888, 512, 512), "dec_ff1": (101888, 2048, 512),
    "dec_ff2": (101888, 512, 2048),
    # ViT-B/16 encoder (D = 768, J = 2304)
    "b_qkv": (26624, 2304, 768), "b_wo": (26624, 768, 768), "b_ff1": (25088, 3072, 768),
    "b_ff2": (25088, 768, 3072), "b_jumbo1": (512, 9216, 2304), "b_jumbo2": (512, 2304, 9216),
    # jumbo MLP at the headline's 2048-image micro-batch
    "jumbo1_2k": (2048, 12288, 3072), "jumbo2_2k": (2048, 3072, 12288),
    # finetune jumbo MLP (128 images)
    "ft_jumbo1": (128, 9216, 2304), "ft_jumbo2": (128, 2304, 9216),
    # ViT-L at the headline's 2048-image micro-batch (52 / 49 encoder rows, 199 decoder rows per image)
    "enc_qkv_2k": (106496, 3072, 1024), "enc_wo_2k": (106496, 1024, 1024), "enc_ff1_2k": (100352, 4096, 1024),
    "enc_ff2_2k": (100352, 1024, 4096), "dec_qkv_2k": (407552, 1536, 512), "dec_wo_2k": (407552, 512, 512),
    "dec_ff1_2k": (407552, 2048, 512), "dec_ff2_2k": (407552, 512, 2048),
    # ViT-B/16 finetune (128 images x 199 tokens; the FF runs on the 196 patch rows = b_ff1/b_ff2)
    "ft_qkv": (25472, 2304, 768), "ft_wo": (25472, 768, 768),
}


def timeit(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def reference(kind, x, w, b, pre):
    """fp32 reference of what ``ours`` computes for each kind (data-gradient kinds carry no bias;
    the dGELU kinds multiply the bf16-rounded GEMM output, as the epilogue does)."""
    base = x.float() @ w.float().t()
    if kind == "dgrad":
        return base
    if kind == "dgrad_gelu":
        h = pre.float()
        t = torch.tanh(0.7978845608028654 * (h + 0.044715 * h ** 3))
        d = 0.5 * (1 + t) + 0.5 * h * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * h * h)
        return base.bfloat16().float() * d
    if kind in ("dgrad_dmul", "dgrad_dmul_nob"):  # pre: the 8-bit gelu' codes (ops/prims.py gd_decode)
        return base.bfloat16().float() * ((pre.float() - P.GD_Z) / P.GD_Q)
    r = base + b
    if kind in ("fwd_gelu_only", "fwd_gelu_d"):
        return torch.nn.functional.gelu(r.bfloat16().float(), approximate="tanh")
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    ap.add_argument("--kinds", default="fwd,fwd_gelu,dgrad")
    ap.add_argument("--variant", default="0", help="kernel path(s) (ext.gemm_test_force), comma separated: 0 = by "
                    "shape, 1 = 64-deep main loop everywhere, 2 = 4-phase kernels at every M without tail split, "
                    "2rNNN = the same at forced tile height NNN (256 / 224 / 192); several = interleaved A/B")
    a = ap.parse_args()
    ext = _ext.load()
    variants = a.variant.split(",")

    def setv(v):
        m = re.search(r"r(\d+)", v)
        ext.gemm_test_force(int(re.sub(r"r\d+", "", v)), int(m.group(1)) if m else 0)

    setv(variants[0])
    names = [n for n in FWD if not a.only or n in a.only.split(",")]
    tot = {"ours": 0.0, "blas": 0.0}
    for kind in a.kinds.split(","):
        for name in names:
            M, N, K = FWD[name]
            if kind.startswith("fwd_gelu") and name not in ("enc_ff1", "dec_ff1", "enc_ff1_2k", "dec_ff1_2k", "jumbo1", "jumbo1_2k", "b_ff1", "b_jumbo1", "ft_jumbo1"):
                continue
            if kind.startswith("dgrad_") and name not in ("enc_ff2", "dec_ff2", "enc_ff2_2k", "dec_ff2_2k", "b_ff2", "jumbo2", "jumbo2_2k", "b_jumbo2", "ft_jumbo2"):
                continue
            if kind == "splitk" and name not in ("jumbo1", "jumbo2", "b_jumbo2", "ft_jumbo2"):
                continue
            if kind.startswith("dgrad"):  # dX[M,K] = dy[M,N] @ W[N,K]  ->  NT with B = W^T [K, N]
                M, N, K = M, K, N
            x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
            w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()
            b = torch.randn(N, device="cuda") * 0.1
            bb = b.bfloat16()
            gelu = kind == "fwd_gelu"
            pre = None
            if kind == "splitk":
                from jumbo_mae_tpu_amd.ops.prims import splitk_plan
                S = max(2, splitk_plan(M, N, K))
                ours = lambda: (ext.gemm_nt_splitk(x, w, b, S),)  # noqa: E731
                blas = lambda: torch.addmm(bb, x, w.t())  # noqa: E731
            elif kind == "dgrad_gelu":
                wm = w.t().contiguous()
                pre = (torch.randn(M, N, device="cuda") * 2).bfloat16()
                dbg = torch.zeros(N, device="cuda")
                ours = lambda: (ext.gemm_nt_dgelu(x, w, pre, dbg),)  # noqa: E731
                blas = lambda: ext.gelu_bwd(pre, x @ wm, dbg)  # noqa: E731
            elif kind in ("dgrad_dmul", "dgrad_dmul_nob"):  # x saved gelu'(h) (training path), +- FF1 bias grad
                wm = w.t().contiguous()
                pre = torch.randint(1, 255, (M, N), device="cuda", dtype=torch.uint8)  # gelu' codes
                pre_bf = ((pre.float() - P.GD_Z) / P.GD_Q).bfloat16()
                dbg = torch.zeros(N, device="cuda") if kind == "dgrad_dmul" else None
                ours = lambda: (ext.gemm_nt_dgelu(x, w, pre, dbg, True),)  # noqa: E731
                blas = lambda: (x @ wm) * pre_bf  # noqa: E731
            elif kind == "dgrad":
                wm = w.t().contiguous()  # W as the model stores it: [N_fwd, K_fwd] = w^T
                ours = lambda: ext.gemm_nt(x, w, None, False)  # noqa: E731
                blas = lambda: x @ wm  # noqa: E731
            elif kind == "fwd_gelu_only":  # one output, gelu(h): the GELU VALU without the second store
                ours = lambda: ext.gemm_nt(x, w, b, True, True)  # noqa: E731
                blas = lambda: torch.nn.functional.gelu(torch.addmm(bb, x, w.t()), approximate="tanh")  # noqa: E731
            elif kind == "fwd_gelu_d":  # two outputs, gelu'(h) and gelu(h) (the training forward)
                ours = lambda: ext.gemm_nt(x, w, b, True, False, True)  # noqa: E731
                blas = lambda: torch.nn.functional.gelu(torch.addmm(bb, x, w.t()), approximate="tanh")  # noqa: E731
            elif gelu:
                ours = lambda: ext.gemm_nt(x, w, b, True)  # noqa: E731
                blas = lambda: torch.nn.functional.gelu(torch.addmm(bb, x, w.t()), approximate="tanh")  # noqa: E731
            else:
                ours = lambda: ext.gemm_nt(x, w, b, False)  # noqa: E731
                blas = lambda: torch.addmm(bb, x, w.t())  # noqa: E731
            ref = reference(kind, x, w, b, pre)
            errs = []
            for v in variants:
                setv(v)
                o = ours()
                if kind == "fwd_gelu_d":
                    o = o[1:]
                errs.append(((o[0].float() - ref).abs().max() / ref.abs().max()).item())
            setv(variants[0])
            out = ours()
            if kind == "fwd_gelu_d":
                out = out[1:]
            err = ((out[0].float() - ref).abs().max() / ref.abs().max()).item()
            if gelu:
                g_ref = torch.nn.functional.gelu(out[0].float(), approximate="tanh")
                err = max(err, ((out[1].float() - g_ref).abs().max() / g_ref.abs().max()).item())
            blas()
            torch.cuda.synchronize()
            tv = {v: [] for v in variants}
            tb = []
            for _ in range(a.rounds):
                for v in variants:
                    setv(v)
                    tv[v].append(timeit(ours, a.iters))
                tb.append(timeit(blas, a.iters))
            setv(variants[0])
            to, tb = min(tv[variants[0]]), min(tb)
            if len(variants) > 1:
                fl = 2.0 * M * N * K
                print("   " + "  ".join(f"v{v}: {min(tv[v]):7.1f} us {fl / min(tv[v]) / 1e6:5.0f} TF err {e:.1e}"
                                        for v, e in zip(variants, errs)), flush=True)
            fl = 2.0 * M * N * K
            tot["ours"] += to
            tot["blas"] += tb
            print(f"{kind:8s} {name:8s} M={M:6d} N={N:5d} K={K:5d}  ours {to:8.1f} us {fl / to / 1e6:6.0f} TF | "
                  f"hipBLASLt {tb:8.1f} us {fl / tb / 1e6:6.0f} TF | x{tb / to:4.2f}  relerr {err:.1e}", flush=True)
    print(f"total ours {tot['ours']:.0f} us  hipBLASLt {tot['blas']:.0f} us")


if __name__ == "__main__":
    main()
