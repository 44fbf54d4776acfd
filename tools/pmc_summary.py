#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc_*/run_counter_collection.csv) per kernel:
median counter value per dispatch, plus HBM bytes per launch with the gfx950 correction
from MI355X_MICROARCH.md (FETCH_SIZE counts half of a wide coalesced read: x2; both
counters are in KiB).  Writes profiles/pmc_summary.json when --write is given."""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAGE = {"k_hist": "hist", "k_colscan": "colscan", "k_scatter": "scatter", "k_scatter_rec": "scatter",
         "k_bounds": "bounds", "k_fold": "fold", "k_fold_wide": "fold", "k_unscatter": "unscatter",
         "k_drain": "drain", "k_hot_plan": "hot", "k_hot_summary": "hot", "k_hot_chain": "hot",
         "k_hot_replies": "hot", "k_hot_update": "hot"}


def our_kernels():
    """Kernel names defined in the engine's HIP sources (torch / rocPRIM kernels of the
    benchmark harness are not part of a step)."""
    names = set()
    for f in glob.glob(os.path.join(ROOT, "distributedratelimiting.redis_amd", "csrc", "*.hip")):
        names.update(re.findall(r"\bvoid\s+(k_\w+)\s*\(", open(f).read()))
    return names


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    m = re.search(r"\b(k_\w+)", n)
    base = m.group(1) if m else n.split("(")[0]
    t = re.search(r"k_\w+<([^>]*)>", n)
    return base + (f"<{t.group(1)}>" if t else "")


def main():
    # gpurun_out/pmc_<workload>_<counter>/ (tools/pmc_all.sh); older pmc_<name>/ dirs count
    # as the uniform workload
    agg = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(list)))
    for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "pmc_*", "run_counter_collection.csv"))):
        tag = os.path.basename(os.path.dirname(f))[4:]
        w = tag.split("_")[0] if tag.split("_")[0] in ("uniform", "zipf", "queue", "approx") else "uniform"
        for r in csv.DictReader(open(f)):
            agg[w][short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    by_w = {}
    for w in sorted(agg):
        out = by_w.setdefault(w, {})
        for k in sorted(agg[w]):
            if not k.startswith("k_"):
                continue
            # median per dispatch: robust to warm-up dispatches (a Zipf run's first batches
            # fold hot keys in their buckets before the hot set exists)
            d = {c: sorted(v)[len(v) // 2] for c, v in agg[w][k].items()}
            d["dispatches"] = max(len(v) for v in agg[w][k].values())
            if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
                d["hbm_bytes_per_launch"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
            out[k] = d
            print(w, k, " ".join(f"{c}={v:.4g}" for c, v in d.items()))
    stages = {}
    for k, d in by_w.get("uniform", {}).items():   # bench.py's stages: the token-bucket path
        st = STAGE.get(k.split("<")[0])
        if st and "hbm_bytes_per_launch" in d:
            e = stages.setdefault(st, {"hbm_bytes_per_launch": 0.0, "kernels": []})
            e["kernels"].append(k)
            e["hbm_bytes_per_launch"] += d["hbm_bytes_per_launch"]
    for st, e in stages.items():
        # the fold is two launches per batch (k_fold_wide: full buckets, k_fold: the rest),
        # summed; other stages are one kernel per pass, averaged over the passes
        if st != "fold":
            e["hbm_bytes_per_launch"] /= len(e["kernels"])
    # whole-step HBM bytes: every pipeline kernel's median bytes per launch times its
    # average launches per batch (dispatches / dispatches of the fold kernel)
    step = {}
    marker = {"uniform": "k_fold_wide<true>", "zipf": "k_fold_wide<true>", "queue": "k_fold_q<true>",
              "approx": "k_fold_a<true>"}
    skip = ("k_gen_batch", "k_init_table", "k_init_approx", "k_count_queued", "k_gen_zipf")
    ours = our_kernels()
    for w, kern in by_w.items():
        m = kern.get(marker.get(w, ""), {}).get("dispatches")
        if not m:
            continue
        tot = 0.0
        for k, d in kern.items():
            if k.split("<")[0] in skip or k.split("<")[0] not in ours or "hbm_bytes_per_launch" not in d:
                continue
            tot += d["hbm_bytes_per_launch"] * d["dispatches"] / m
        step[w] = round(tot, 1)
        print(w, "step HBM bytes", f"{tot:.4g}")
    if "--write" in sys.argv:
        with open(os.path.join(ROOT, "profiles", "pmc_summary.json"), "w") as f:
            json.dump({"note": "per-launch medians; HBM bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB "
                               "(gfx950 FETCH_SIZE correction, MI355X_MICROARCH.md HBM section); "
                               "stages = the token-bucket (uniform) path",
                       **stages, "step_hbm_bytes": step, "kernels": by_w.get("uniform", {}),
                       "workloads": by_w}, f, indent=1)


if __name__ == "__main__":
    main()
