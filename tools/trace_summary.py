import csv, re, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1]))); steps = int(sys.argv[2]); pat = sys.argv[3] if len(sys.argv) > 3 else ""
agg = defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    m = re.search(r"::(\w+(<[^()]*>)?)\(", n)
    short = m.group(1) if m else n[:60]
    if pat and not re.search(pat, n): continue
    key = (short[:60], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), r["VGPR_Count"], r["LDS_Block_Size"])
    agg[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:40]:
    print(f"{sum(v)/1e6/steps:7.3f} ms/step n={len(v)//steps:4d} avg={sum(v)/len(v)/1e3:8.1f}us  blocks={k[1]:7d} vgpr={k[2]} lds={k[3]} {k[0]}")
