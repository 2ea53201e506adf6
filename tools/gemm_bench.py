"""Time every GEMM of the ViT-L jumbo-MAE step (B=512/GPU) through hipBLASLt (torch) on the box."""
import torch, time, json, sys
torch.backends.cuda.matmul.allow_tf32 = False
dev = "cuda"
B = 512
E = B * 52; P = B * 49; C = B; DM = B * 199; PR = B * 196
D, J, d = 1024, 3072, 512
# (name, M, N, K, count per step)
shapes = [
  ("enc_qkv", E, 3*D, D, 24), ("enc_wo", E, D, D, 24), ("enc_ff1", P, 4*D, D, 24), ("enc_ff2", P, D, 4*D, 24),
  ("jumbo1", C, 4*J, J, 24), ("jumbo2", C, J, 4*J, 24),
  ("dec_qkv", DM, 3*d, d, 8), ("dec_wo", DM, d, d, 8), ("dec_ff1", DM, 4*d, d, 8), ("dec_ff2", DM, d, 4*d, 8),
  ("patch", P, D, 768, 1), ("dproj", E, d, D, 1), ("pred", PR, 768, d, 1),
]
def timeit(fn, n=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / n
res = []; tot = {"fwd": 0, "dgrad": 0, "wgrad": 0, "wgrad_bf16": 0}
for name, M, N, K, cnt in shapes:
    x = torch.randn(M, K, device=dev).bfloat16(); w = torch.randn(N, K, device=dev).bfloat16() * 0.02
    b = torch.randn(N, device=dev).bfloat16(); dy = torch.randn(M, N, device=dev).bfloat16()
    g = torch.zeros(N, K, device=dev)
    f = 2 * M * N * K
    t_f = timeit(lambda: torch.addmm(b, x, w.t()))
    t_d = timeit(lambda: dy @ w)
    t_w = timeit(lambda: torch.addmm(g, dy.t(), x, out_dtype=torch.float32, out=g))
    t_w2 = timeit(lambda: dy.t() @ x)
    for k, t in (("fwd", t_f), ("dgrad", t_d), ("wgrad", t_w), ("wgrad_bf16", t_w2)): tot[k] += t * cnt
    r = dict(name=name, M=M, N=N, K=K, fwd_tf=f / t_f / 1e12, dgrad_tf=f / t_d / 1e12, wgrad_tf=f / t_w / 1e12,
             wgrad_bf16_tf=f / t_w2 / 1e12, ms_step=(t_f + t_d + t_w) * cnt * 1e3)
    res.append(r); print(json.dumps(r), flush=True)
    del x, w, b, dy, g
print("per-step totals ms:", {k: round(v * 1e3, 2) for k, v in tot.items()})
