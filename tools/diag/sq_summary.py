"""Diagnostic (round 6): mean per dispatch of each SQ counter of the kernels whose name
contains a substring, from a rocprofv3 --pmc counter_collection CSV (tools/diag/sq_pass.sh),
with per-wave instruction counts.
usage: python tools/diag/sq_summary.py <run_counter_collection.csv> <kernel substring>"""
import csv
import sys
from collections import defaultdict


def main():
    path, sub = sys.argv[1], sys.argv[2]
    per = defaultdict(lambda: defaultdict(float))   # dispatch -> counter -> value (summed over dims)
    names = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if sub not in r["Kernel_Name"]:
                continue
            d = r["Dispatch_Id"]
            names[d] = r["Kernel_Name"]
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        print("no dispatch of", sub)
        return
    tot = defaultdict(float)
    for d in per.values():
        for k, v in d.items():
            tot[k] += v
    n = len(per)
    print(f"{sub}: {n} dispatches ({sorted(set(names.values()))[0][:80]})")
    for k in sorted(tot):
        print(f"  {k:<20} {tot[k] / n:16.1f}")
    w = tot.get("SQ_WAVES", 0.0)
    if w:
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM"):
            if k in tot:
                print(f"  {k} per wave {tot[k] / w:10.1f}")


if __name__ == "__main__":
    main()
