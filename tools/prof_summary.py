import csv, sys
path = sys.argv[1]; steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
cat = {}
for r in rows:
    n = r["Name"]; t = float(r["TotalDurationNs"]) / 1e6 / steps
    if n.startswith("Cijk") or n.startswith("Custom_Cijk"): k = "GEMM(hipBLASLt)"
    elif "gemm_" in n: k = "GEMM (ours, MFMA)"
    elif "attn" in n: k = "attention"
    elif any(x in n for x in ("patch", "unshuffle", "embed_finish")): k = "mae glue (ours)"
    elif "ln_" in n: k = "layernorm"
    elif "rowcol" in n or "gelu" in n or "residual" in n or "splitk" in n or "transpose_bf16" in n: k = "fused elementwise (ours)"
    elif "adamw" in n or "opt" in n.lower() or "sumsq" in n: k = "optimizer"
    elif "at::native" in n: k = "torch native"
    else: k = "other"
    cat[k] = cat.get(k, 0) + t
print(f"total {tot/1e6/steps:.2f} ms/step (incl. init kernels)")
for k, v in sorted(cat.items(), key=lambda x: -x[1]): print(f"  {k:28s} {v:8.2f} ms/step")
print()
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f'{float(r["TotalDurationNs"])/1e6/steps:8.3f} ms  n={int(r["Calls"])//steps:5d}  {r["Name"][:100]}')
