"""One training step's kernel timeline from a rocprofv3 kernel_trace.csv (step = the kernels
between two consecutive optimizer launches): busy vs wall time, idle gaps, and per-kernel rows.

    python tools/step_timeline.py gpurun_out/prof/run_kernel_trace.csv [--step -2] [--top 40]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--step", type=int, default=-2, help="which step (index among optimizer launches)")
    ap.add_argument("--top", type=int, default=0, help="print the N longest kernels of the step")
    ap.add_argument("--all", action="store_true", help="print every kernel of the step in order")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    opt = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
    i0, i1 = opt[a.step - 1] + 1, opt[a.step] + 1
    step = rows[i0:i1]
    t0 = int(step[0]["Start_Timestamp"])
    t1 = int(step[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
    gaps = []
    for p, q in zip(step, step[1:]):
        g = int(q["Start_Timestamp"]) - int(p["End_Timestamp"])
        if g > 0:
            gaps.append((g, p["Kernel_Name"][:50], q["Kernel_Name"][:50]))
    print(f"kernels {len(step)}  wall {(t1 - t0) / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  "
          f"idle {sum(g for g, _, _ in gaps) / 1e6:.2f} ms in {len(gaps)} gaps")
    for g, p, q in sorted(gaps, reverse=True)[:8]:
        print(f"   gap {g / 1e3:8.1f} us  after {p}  before {q}")
    if a.all or a.top:
        lst = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), (int(r["Start_Timestamp"]) - t0) / 1e3,
                r["Kernel_Name"][:90], r["Grid_Size_X"], r["Workgroup_Size_X"]) for r in step]
        if a.top:
            lst = sorted(lst, reverse=True)[:a.top]
        for d, s, n, gx, wx in lst:
            print(f"{s:10.1f} us  {d / 1e3:8.1f} us  grid {int(gx) // max(1, int(wx)):6d}  {n}")


if __name__ == "__main__":
    main()
