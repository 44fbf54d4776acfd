#!/usr/bin/env python3
"""Print a rocprofv3 --stats kernel summary compactly: python tools/prof_stats.py <kernel_stats.csv>"""
import csv
import re
import sys

for r in csv.DictReader(open(sys.argv[1])):
    n = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", ""))
    print(f'{n[:58]:58s} calls={r["Calls"]:>4s} avg_us={float(r["AverageNs"]) / 1e3:9.1f} '
          f'min_us={float(r["MinNs"]) / 1e3:9.1f} total_ms={float(r["TotalDurationNs"]) / 1e6:8.2f}')
