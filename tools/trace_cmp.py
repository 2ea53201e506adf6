"""Compare two rocprofv3 kernel traces of the flagship step (e.g. plain vs 1-rank RCCL DP):
per-step wall, summed kernel time, busy-interval union (overlap-aware) and the kernels whose
per-step time differs most.  Steps are delimited by patch_mse_fwd (once per pretrain step).

    python tools/trace_cmp.py A/run_kernel_trace.csv B/run_kernel_trace.csv
"""
import csv, sys, collections
def load(p):
    rows = sorted(csv.DictReader(open(p)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "patch_mse_fwd" in r["Kernel_Name"]]
    # last 4 full steps
    a, b = idx[-5], idx[-1]
    step = rows[a:b]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    per = collections.defaultdict(lambda: [0, 0])
    busy = 0
    for r in step:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        k = r["Kernel_Name"][:70]
        per[k][0] += d; per[k][1] += 1
        busy += d
    # union of busy intervals (overlap-aware)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step)
    u = 0; cs, ce = iv[0]
    for s, e in iv[1:]:
        if s > ce: u += ce - cs; cs, ce = s, e
        else: ce = max(ce, e)
    u += ce - cs
    return (t1 - t0) / 4e6, busy / 4e6, u / 4e6, {k: (v[0] / 4e3, v[1] / 4) for k, v in per.items()}, len(step) / 4
A = load(sys.argv[1]); B = load(sys.argv[2])
print(f"plain: wall {A[0]:.2f} ms/step busy-sum {A[1]:.2f} union {A[2]:.2f} kernels {A[4]}")
print(f"dp64 : wall {B[0]:.2f} ms/step busy-sum {B[1]:.2f} union {B[2]:.2f} kernels {B[4]}")
keys = set(A[3]) | set(B[3])
diff = sorted(keys, key=lambda k: -abs(B[3].get(k, (0, 0))[0] - A[3].get(k, (0, 0))[0]))
for k in diff[:25]:
    a = A[3].get(k, (0, 0)); b = B[3].get(k, (0, 0))
    print(f"{b[0]-a[0]:+9.1f} us  plain {a[0]:9.1f} us x{a[1]:6.1f}  dp {b[0]:9.1f} us x{b[1]:6.1f}  {k}")
