"""Per-step kernel summary from a rocprofv3 kernel trace, steady-state steps only.

    python tools/trace_steps.py <run_kernel_trace.csv> [--last N] [--top K] [--marker adamw_kernel]

Steps are delimited by the optimizer kernel (``--marker``, one launch per step); the warmup steps
and the model-initialisation kernels before the first marker are excluded, which
``prof_summary.py`` (whole-trace totals / steps) cannot do.  Prints ms/step per category (same
categories as prof_summary.py), the busy time, the wall time between markers, and the top kernels
with calls per step."""

import argparse
import collections
import csv


def category(n: str) -> str:
    if n.startswith("Cijk") or n.startswith("Custom_Cijk"):
        return "GEMM (hipBLASLt)"
    if "gemm_" in n:
        return "GEMM (ours, MFMA)"
    if "attn" in n:
        return "attention"
    if any(x in n for x in ("patch", "unshuffle", "embed_finish", "mask_ids", "gather_patches")):
        return "mae glue (ours)"
    if "ln_" in n:
        return "layernorm"
    if any(x in n for x in ("rowcol", "gelu", "residual", "splitk", "colsum", "transpose_bf16", "zero_")):
        return "fused elementwise (ours)"
    if "adamw" in n or "opt" in n.lower() or "sumsq" in n or "lamb" in n or "lars" in n or "chunk_sums" in n:
        return "optimizer"
    if "at::native" in n:
        return "torch native"
    if "rocclr" in n:
        return "runtime copies / fills"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=4)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--marker", default="adamw_kernel")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(marks) < 2:
        raise SystemExit(f"fewer than two '{a.marker}' launches in the trace")
    pairs = list(zip(marks[:-1], marks[1:]))[-a.last:]
    cat = collections.Counter()
    kt = collections.Counter()
    kn = collections.Counter()
    busy = wall = 0.0
    for lo, hi in pairs:
        seg = rows[lo + 1:hi + 1]
        wall += (int(rows[hi]["End_Timestamp"]) - int(rows[lo]["End_Timestamp"])) / 1e6
        for r in seg:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            n = r["Kernel_Name"]
            busy += d
            cat[category(n)] += d
            kt[n] += d
            kn[n] += 1
    ns = len(pairs)
    print(f"{ns} steady-state steps: wall {wall / ns:.2f} ms/step, kernel busy {busy / ns:.2f} ms/step")
    for k, v in cat.most_common():
        print(f"  {k:28s} {v / ns:8.3f} ms/step")
    print()
    for n, v in kt.most_common(a.top):
        print(f"{v / ns:8.3f} ms  {kn[n] / ns:6.1f}/step  {n[:110]}")


if __name__ == "__main__":
    main()
