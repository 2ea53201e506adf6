"""Per-launch-shape totals of the GEMM kernels in a rocprofv3 kernel trace: kernel, workgroups,
calls per step, mean us, and (for 256 x 256 launches) the wave count -- to price tile
quantisation (a last wave that fills part of the 256 CUs).

    python tools/trace_gemm.py gpurun_out/<run>/prof/run_kernel_trace.csv [steps]
"""
import collections
import csv
import re
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        m = re.search(r"(gemm_\w+|tail_finish_kernel|splitk_reduce\w*)(<[^>(]*>)?", name)
        if not m:
            continue
        wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        agg[(m.group(0), wg)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    if not steps:
        steps = max(len(v) for v in agg.values()) // 24 or 1
    tot = 0.0
    out = []
    for (k, wg), v in agg.items():
        s = sum(v) / steps
        tot += s
        out.append((s, k, wg, len(v) / steps, sum(v) / len(v)))
    out.sort(reverse=True)
    print(f"{'kernel':34s} {'WGs':>6s} {'waves':>6s} {'calls/step':>10s} {'mean us':>9s} {'ms/step':>8s}")
    for s, k, wg, c, mu in out:
        print(f"{k:34s} {wg:6d} {wg / 256:6.2f} {c:10.1f} {mu:9.1f} {s / 1e3:8.3f}")
    print(f"total {tot / 1e3:.2f} ms/step over {steps} steps")


if __name__ == "__main__":
    main()
