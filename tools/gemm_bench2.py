"""wgrad alternatives: layouts, rocBLAS vs hipBLASLt, TunableOp."""
import os, sys, time, json
mode = sys.argv[1]
if mode == "tunable":
    os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
    os.environ["PYTORCH_TUNABLEOP_TUNING"] = "1"
    os.environ["PYTORCH_TUNABLEOP_FILENAME"] = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "tunableop_results%d.csv")
    os.environ["PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS"] = "60"
import torch
if mode == "rocblas":
    torch.backends.cuda.preferred_blas_library("cublas")
B = 512
E = B * 52; P = B * 49; C = B; DM = B * 199
D, J, d = 1024, 3072, 512
shapes = [("enc_qkv", E, 3*D, D, 24), ("enc_wo", E, D, D, 24), ("enc_ff1", P, 4*D, D, 24), ("enc_ff2", P, D, 4*D, 24),
  ("jumbo1", C, 4*J, J, 24), ("jumbo2", C, J, 4*J, 24), ("dec_qkv", DM, 3*d, d, 8), ("dec_wo", DM, d, d, 8),
  ("dec_ff1", DM, 4*d, d, 8), ("dec_ff2", DM, d, 4*d, 8)]
def timeit(fn, n=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / n
tot = {}
for name, M, N, K, cnt in shapes:
    x = torch.randn(M, K, device="cuda").bfloat16(); dy = torch.randn(M, N, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16(); b = torch.randn(N, device="cuda").bfloat16()
    f = 2 * M * N * K
    r = {"name": name}
    cands = {
        "w_TN_bf16": lambda: dy.t() @ x,
        "w_NT_bf16": lambda: x.t() @ dy,
        "w_TN_f32": lambda: torch.mm(dy.t(), x, out_dtype=torch.float32),
        "fwd": lambda: torch.addmm(b, x, w.t()),
        "dgrad": lambda: dy @ w,
    }
    for k, fn in cands.items():
        try:
            t = timeit(fn); r[k] = round(f / t / 1e12, 1); tot[k] = tot.get(k, 0) + t * cnt * 1e3
        except Exception as e:
            r[k] = str(e)[:60]
    print(json.dumps(r), flush=True)
print(mode, "per-step ms:", {k: round(v, 2) for k, v in tot.items()}, flush=True)
