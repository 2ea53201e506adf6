"""Does the input pipeline overlap the train step?  From a rocprofv3 trace of the pretrain driver
(``--kernel-trace --memory-copy-trace``), over the steady-state steps (between the last
``--last`` + 1 optimizer launches):

* host->device copies: total time, and the part that runs while a model kernel runs (overlapped);
* device-augment kernels (``rrc_h_kernel`` / ``rrc_v_kernel``): total time, and the part that runs
  beside a model kernel (on the prefetch stream) rather than alone;
* GPU idle time between the steps' kernels (gaps > ``--gap-us``): host syncs or data stalls show
  up here.

    python tools/overlap_check.py <kernel_trace.csv> <memory_copy_trace.csv> [--last 8]
"""

from __future__ import annotations

import argparse
import csv
import json


def _iv(rows):
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)


def _merge(ivs):
    out = []
    for a, b in sorted(ivs):
        if out and a <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], b))
        else:
            out.append((a, b))
    return out


def _overlap(ivs, cover):
    """Total length of ``ivs`` covered by the merged intervals ``cover``."""
    tot, j = 0, 0
    for a, b in ivs:
        while j < len(cover) and cover[j][1] <= a:
            j += 1
        k = j
        while k < len(cover) and cover[k][0] < b:
            tot += max(0, min(b, cover[k][1]) - max(a, cover[k][0]))
            k += 1
    return tot


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("kernels")
    ap.add_argument("copies")
    ap.add_argument("--last", type=int, default=8)
    ap.add_argument("--marker", default="adamw_kernel")
    ap.add_argument("--gap-us", type=float, default=20.0)
    a = ap.parse_args(argv)
    ks = list(csv.DictReader(open(a.kernels)))
    cs = list(csv.DictReader(open(a.copies)))
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [int(r["Start_Timestamp"]) for r in ks if a.marker in r["Kernel_Name"]]
    if len(marks) < a.last + 1:
        raise SystemExit(f"only {len(marks)} '{a.marker}' launches")
    t0, t1 = marks[-a.last - 1], marks[-1]
    inside = lambda r: t0 <= int(r["Start_Timestamp"]) < t1  # noqa: E731
    ks = [r for r in ks if inside(r)]
    aug = [r for r in ks if "rrc_" in r["Kernel_Name"]]
    model = [r for r in ks if "rrc_" not in r["Kernel_Name"]]
    dirs = [r for r in cs if inside(r)]
    h2d = [r for r in dirs if "HOST_TO_DEVICE" in r.get("Direction", "").upper() or "H2D" in r.get("Direction", "").upper()]
    mcov = _merge(_iv(model))
    h2d_t = sum(b - a for a, b in _iv(h2d))
    aug_t = sum(b - a for a, b in _iv(aug))
    allcov = _merge(_iv(ks))
    gaps = [(b0, a1) for (_, b0), (a1, _) in zip(allcov, allcov[1:]) if a1 - b0 > a.gap_us * 1e3]
    steps = a.last
    out = {"steps": steps, "step_ms": (t1 - t0) / steps / 1e6,
           "model_kernel_busy_ms_per_step": sum(b - a for a, b in mcov) / steps / 1e6,
           "h2d_copies_per_step": len(h2d) / steps, "h2d_ms_per_step": h2d_t / steps / 1e6,
           "h2d_overlapped_frac": _overlap(_iv(h2d), mcov) / h2d_t if h2d_t else None,
           "augment_kernels_per_step": len(aug) / steps, "augment_ms_per_step": aug_t / steps / 1e6,
           "augment_overlapped_frac": _overlap(_iv(aug), mcov) / aug_t if aug_t else None,
           f"idle_gaps_over_{a.gap_us:g}us_per_step": len(gaps) / steps,
           "idle_ms_per_step": sum(b - a for a, b in gaps) / steps / 1e6}
    print(json.dumps(out))
    return out


if __name__ == "__main__":
    main()
