"""wgrad via batched split-K (bmm over M-chunks, fp32 out) + reduction, vs plain."""
import torch, time, json
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
    g = torch.zeros(N, K, device="cuda")
    f = 2 * M * N * K
    r = {"name": name}
    def plain(): torch.addmm(g, dy.t(), x, out_dtype=torch.float32, out=g)
    cands = {"plain": plain}
    for S in (2, 4, 8, 16):
        if M % S: continue
        Mc = M // S
        buf = torch.empty(S, N, K, device="cuda")
        def split(S=S, Mc=Mc, buf=buf):
            torch.bmm(dy.view(S, Mc, N).transpose(1, 2), x.view(S, Mc, K), out_dtype=torch.float32, out=buf)
            g.add_(buf.sum(0))
        def split_bf(S=S, Mc=Mc):
            t = torch.bmm(dy.view(S, Mc, N).transpose(1, 2), x.view(S, Mc, K))
            g.add_(t.sum(0, dtype=torch.float32))
        cands[f"split{S}"] = split
        cands[f"splitbf{S}"] = split_bf
    for k, fn in cands.items():
        try:
            t = timeit(fn); r[k] = round(f / t / 1e12, 1); tot[k] = tot.get(k, 0) + t * cnt * 1e3
        except Exception as e:
            r[k] = str(e)[:80]
    print(json.dumps(r), flush=True)
print("per-step ms:", {k: round(v, 2) for k, v in tot.items()}, flush=True)
