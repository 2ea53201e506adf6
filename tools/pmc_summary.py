"""Summarise rocprofv3 --pmc counter_collection.csv files: mean counter value per dispatch,
grouped by kernel (name prefix).

    python tools/pmc_summary.py gpurun_out/apmc1/run_counter_collection.csv [more.csv ...]
"""
import collections
import csv
import sys


def main():
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"][:70]
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add((path, r["Dispatch_Id"]))
    for k, cs in per.items():
        print(k)
        for c, v in sorted(cs.items()):
            n = len(disp[(k, c)])
            print(f"    {c:28s} {v / n:16.1f}")


if __name__ == "__main__":
    main()
