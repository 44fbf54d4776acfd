#!/usr/bin/env python3
"""Per-kernel durations of a rocprofv3 --kernel-trace run of bench.py, restricted to marker
windows (include/tbe_tools.h tbe_mark_device):

  timed   dispatches enqueued between k_mark<1> and k_mark<2>: the pipelined timed batches
  replay  between k_mark<3> and k_mark<4>: the serial replay of the same batches, whose
          HIP-event stage times give the bench line's roofline (avg_launch_ms)

so that `frac` can be recomputed from profiles/ alone, without the warm-up batches (the
first two Zipf batches run before any hot key is nominated: their fold takes ~27 ms) or
the legs after the timed region.  Usage:
    python tools/prof_window.py <run_kernel_trace.csv> [--out profiles/<name>.json]"""
import argparse
import collections
import csv
import json
import re
import statistics


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    m = re.search(r"\b(k_\w+(<[^()]*>)?)", n)
    return m.group(1) if m else n.split("(")[0][:60]


def windows(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    marks = {}
    for r in rows:
        m = re.search(r"k_mark<(\d)>", r["Kernel_Name"])
        if m:
            marks.setdefault(int(m.group(1)), int(r["Dispatch_Id"]))
    out = {}
    for name, (a, b) in (("timed", (1, 2)), ("replay", (3, 4))):
        if a not in marks or b not in marks:
            continue
        per = collections.defaultdict(list)
        for r in rows:
            d = int(r["Dispatch_Id"])
            if marks[a] < d < marks[b] and "k_mark" not in r["Kernel_Name"]:
                per[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        out[name] = {k: {"calls": len(v), "avg_us": round(statistics.mean(v), 2), "min_us": round(min(v), 2),
                         "max_us": round(max(v), 2), "total_us": round(sum(v), 1)}
                     for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))}
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out")
    a = ap.parse_args()
    res = windows(a.trace)
    for w, ks in res.items():
        print(f"== {w}")
        for k, v in ks.items():
            print(f"  {k[:60]:60s} calls={v['calls']:4d} avg_us={v['avg_us']:9.2f} min={v['min_us']:9.2f} max={v['max_us']:9.2f}")
    if a.out:
        json.dump({"trace": a.trace, "windows": res}, open(a.out, "w"), indent=1)
