#!/usr/bin/env python3
"""Per-kernel summary of an SQ-counter pass (tools/pmc_sq.sh, tools/pmc_sq_var.sh):
python tools/sq_summary.py gpurun_out/pmcsq_<name>/run_counter_collection.csv"""
import collections
import csv
import re
import statistics
import sys

for path in sys.argv[1:]:
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))
        d[(n, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for (n, _), cs in d.items():
        for c, v in cs.items():
            agg[n][c].append(v)
    print("==", path)
    for n, cs in agg.items():
        if "k_" not in n:
            continue
        m = {c: statistics.median(v) for c, v in cs.items()}
        wc = m.get("SQ_WAVE_CYCLES", 1) or 1
        print(f"{n[:44]:44s} wave_cyc={wc:.3g} wait={m['SQ_WAIT_ANY']/wc:.2f} instwait={m['SQ_WAIT_INST_ANY']/wc:.2f} "
              f"active={m['SQ_ACTIVE_INST_ANY']/wc:.2f} valu={m['SQ_INSTS_VALU']:.3g} lds={m['SQ_INSTS_LDS']:.3g} "
              f"bankc={m['SQ_LDS_BANK_CONFLICT']:.3g}")
