#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of tools/pmc_passes.sh into profiles/pmc_summary.json.

* Calibration (gpurun_out/pmc3_calib_p*/): the k_calib<mode> dispatches move known byte
  counts (tools/pmc_calib.py).  For each byte model below the summary reports counted /
  known bytes per pattern, and picks for reads and for writes the model that counts the
  streaming patterns (16, 8 and 4 B per lane) closest to their true bytes.  Read models:
    fetch      FETCH_SIZE * 1 KiB                       (raw)
    fetch_x2   2 * FETCH_SIZE * 1 KiB                   (MI355X_MICROARCH.md: wide streams)
    requests   128 * RDREQ_128B + 64 * RDREQ_64B + 32 * RDREQ_32B
    dram32     32 * TCC_EA0_RDREQ_DRAM_32B              (32-byte sectors sent to DRAM)
  Write models: write_size (WRITE_SIZE * 1 KiB), dram32 (32 * TCC_EA0_WRREQ_WRITE_DRAM_32B).
* Workloads (gpurun_out/pmc3_<workload>_p*/, bench.py --steps 20 --warmup 5 as the driver
  runs it): only the dispatches enqueued between the k_mark<1> and k_mark<2> markers --
  the 20 timed batches -- count.  Per kernel: the chosen models' bytes per launch (mean
  over the timed launches) and per step; per workload: the step's total.

Writes profiles/pmc_summary.json with --write."""
import collections
import csv
import glob
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
STEPS = 20
WIDTH = {0: 16, 1: 8, 2: 4, 3: 16, 4: 8, 5: 4, 6: 16, 7: 4, 8: 16, 9: 1}
STREAM = 1 << 30
GATHER_N = 1 << 23


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    m = re.search(r"\b(k_\w+)", n)
    base = m.group(1) if m else n.split("(")[0]
    t = re.search(r"k_\w+<([^>]*)>", n)
    return base + (f"<{t.group(1)}>" if t else "")


def load(run):
    """{dispatch id: (kernel, {counter: value}, duration ns)} over every pass of `run`."""
    disp = {}
    for f in sorted(glob.glob(os.path.join(OUT, f"pmc3_{run}_p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            p = os.path.basename(os.path.dirname(f))
            key = (p, int(r["Dispatch_Id"]))
            k, c, d = disp.setdefault(key, (short(r["Kernel_Name"]), {}, int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return disp


def windows(disp):
    """Per pass, the dispatch ids strictly between k_mark<1> and k_mark<2> (whole run if
    the markers are absent)."""
    by_pass = collections.defaultdict(list)
    for (p, i), (k, c, d) in disp.items():
        by_pass[p].append((i, k, c, d))
    out = {}
    for p, rows in by_pass.items():
        rows.sort()
        lo = next((i for i, k, _, _ in rows if k == "k_mark<1>"), None)
        hi = next((i for i, k, _, _ in rows if k == "k_mark<2>"), None)
        out[p] = [(k, c, d) for i, k, c, d in rows
                  if (lo is None or i > lo) and (hi is None or i < hi) and not k.startswith("k_mark")]
    return out


def merge(rows_by_pass):
    """kernel -> {counter: [per-dispatch values]} (every pass runs the same dispatches)."""
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for p, rows in rows_by_pass.items():
        for k, c, d in rows:
            for name, v in c.items():
                agg[k][name].append(v)
            if p.endswith("_p0"):
                dur[k].append(d)
    return agg, dur


def read_models(c):
    m = {}
    if "FETCH_SIZE" in c:
        m["fetch"] = c["FETCH_SIZE"] * 1024
        m["fetch_x2"] = 2 * c["FETCH_SIZE"] * 1024
    if all(x in c for x in ("TCC_EA0_RDREQ_128B", "TCC_EA0_RDREQ_64B", "TCC_EA0_RDREQ_32B")):
        m["requests"] = 128 * c["TCC_EA0_RDREQ_128B"] + 64 * c["TCC_EA0_RDREQ_64B"] + 32 * c["TCC_EA0_RDREQ_32B"]
    if "TCC_EA0_RDREQ_DRAM_32B" in c:
        m["dram32"] = 32 * c["TCC_EA0_RDREQ_DRAM_32B"]
    return m


def write_models(c):
    m = {}
    if "WRITE_SIZE" in c:
        m["write_size"] = c["WRITE_SIZE"] * 1024
    if "TCC_EA0_WRREQ_WRITE_DRAM_32B" in c:
        m["dram32"] = 32 * c["TCC_EA0_WRREQ_WRITE_DRAM_32B"]
    return m


def calibrate():
    disp = load("calib")
    if not disp:
        return None
    agg, _ = merge(windows(disp))
    pats = {}
    for m, w in WIDTH.items():
        k = f"k_calib<{m}>"
        if k not in agg:
            continue
        c = {name: statistics.median(v) for name, v in agg[k].items()}
        streaming = m in (0, 1, 2, 6, 7)
        n = STREAM // w if streaming else GATHER_N
        known = n * w
        models = read_models(c) if m <= 5 else write_models(c)
        pats[m] = {"kind": "read" if m <= 5 else "write", "pattern": "stream" if streaming else "scatter",
                   "width": w, "n": n, "known_bytes": known, "counters": c,
                   "model_over_known": {name: round(v / known, 4) for name, v in models.items()},
                   "model_bytes_per_access": {name: round(v / n, 2) for name, v in models.items()}}

    def pick(kind, modes):
        cands = collections.defaultdict(list)
        for m in modes:
            if m in pats:
                for name, r in pats[m]["model_over_known"].items():
                    cands[name].append(abs(r - 1.0))
        full = {n: max(v) for n, v in cands.items() if len(v) == len([m for m in modes if m in pats])}
        return min(full, key=full.get) if full else None

    return {"patterns": pats, "read_model": pick("read", (0, 1, 2)), "write_model": pick("write", (6, 7)),
            "rule": "per direction, the model whose worst error over the streaming patterns (16/8/4 B per "
                    "lane, known bytes) is smallest"}


def summarise(workload, rmodel, wmodel):
    disp = load(workload)
    if not disp:
        return None
    agg, dur = merge(windows(disp))
    kern = {}
    step = {"read": 0.0, "write": 0.0}
    for k, cs in sorted(agg.items()):
        if not k.startswith("k_"):
            continue
        launches = max(len(v) for v in cs.values())
        tot = {name: sum(v) for name, v in cs.items()}
        r = read_models(tot).get(rmodel)
        w = write_models(tot).get(wmodel)
        e = {"launches": launches, "launches_per_step": launches / STEPS,
             "counters_per_launch": {name: v / launches for name, v in tot.items()}}
        if dur.get(k):
            e["pmc_run_avg_ms"] = round(statistics.mean(dur[k]) / 1e6, 4)
        if r is not None and w is not None:
            e["read_bytes_per_launch"] = r / launches
            e["write_bytes_per_launch"] = w / launches
            e["hbm_bytes_per_launch"] = (r + w) / launches
            e["hbm_bytes_per_step"] = (r + w) / STEPS
            step["read"] += r / STEPS
            step["write"] += w / STEPS
        kern[k] = e
    return {"kernels": kern, "step_read_bytes": step["read"], "step_write_bytes": step["write"],
            "step_hbm_bytes": step["read"] + step["write"]}


STAGES = {"k_hist": "hist", "k_hist_dig": "hist", "k_unrank": "unscatter", "k_bscan": "bounds", "k_colscan": "colscan", "k_scatter": "scatter", "k_scatter_rec": "scatter",
          "k_bounds": "bounds", "k_fold": "fold", "k_fold_wide": "fold", "k_fold_q": "fold", "k_fold_a": "fold",
          "k_unscatter": "unscatter", "k_drain": "drain", "k_hot_plan": "hot", "k_hot_summary": "hot",
          "k_hot_chain": "hot", "k_hot_replies": "hot", "k_hot_update": "hot"}


def stage_bytes(w):
    """bench.py's stages: bytes per step and per launch of the stage's kernels."""
    out = {}
    for k, e in w["kernels"].items():
        st = STAGES.get(k.split("<")[0])
        if st and "hbm_bytes_per_step" in e:
            s = out.setdefault(st, {"hbm_bytes_per_step": 0.0, "launches_per_step": 0.0, "kernels": []})
            s["hbm_bytes_per_step"] += e["hbm_bytes_per_step"]
            s["launches_per_step"] += e["launches_per_step"]
            s["kernels"].append(k)
    for s in out.values():
        s["hbm_bytes_per_launch"] = s["hbm_bytes_per_step"] / max(s["launches_per_step"], 1e-9)
    return out


def main():
    cal = calibrate()
    prev = os.path.join(ROOT, "profiles", "pmc_summary.json")
    old = {}
    if os.path.exists(prev):
        with open(prev) as f:
            old = json.load(f)
    if cal is None:   # calibration not rerun: the committed one stands
        cal = old.get("calibration")
    rmodel = (cal or {}).get("read_model") or "fetch_x2"
    wmodel = (cal or {}).get("write_model") or "write_size"
    res = {"note": "rocprofv3 --pmc passes of tools/pmc_passes.sh; workloads ran bench.py --steps 20 --warmup 5 "
                   "and only the dispatches between the k_mark<1>/k_mark<2> markers (the 20 timed batches) "
                   f"count; read bytes by the '{rmodel}' model, write bytes by '{wmodel}' (chosen by the "
                   "calibration patterns, see 'calibration')",
           "read_model": rmodel, "write_model": wmodel, "calibration": cal, "workloads": {}}
    # workloads whose passes are not in this gpurun_out keep their earlier entries (each entry
    # carries the fingerprint of the run it measured; bench.py matches on it)
    res["workloads"].update(old.get("workloads", {}))
    for wl in ("uniform", "zipf", "queue", "approx", "queue_draining"):
        w = summarise(wl, rmodel, wmodel)
        if w:
            w["stages"] = stage_bytes(w)
            # the configuration the passes ran (bench.py writes it under TBE_PMC_FINGERPRINT);
            # bench.py attaches these bytes only to a run with the same fingerprint
            fpath = os.path.join(OUT, f"pmc3_{wl}_fingerprint.json")
            if os.path.exists(fpath):
                with open(fpath) as f:
                    w["fingerprint"] = json.load(f)
            res["workloads"][wl] = w
            print(wl, f"step HBM {w['step_hbm_bytes'] / 1e9:.3f} GB (read {w['step_read_bytes'] / 1e9:.3f}, "
                      f"write {w['step_write_bytes'] / 1e9:.3f})")
            for k, e in w["kernels"].items():
                if "hbm_bytes_per_launch" in e:
                    print(f"   {k:45s} {e['launches_per_step']:5.2f}/step {e['hbm_bytes_per_launch'] / 1e9:8.4f} GB/launch"
                          f" {e.get('pmc_run_avg_ms', 0):8.4f} ms")
    if cal:
        print("calibration: read model", rmodel, "write model", wmodel)
        for m, p in cal["patterns"].items():
            print(f"   mode {m} {p['kind']:5s} {p['pattern']:7s} {p['width']:2d} B/lane ", p["model_over_known"],
                  "per access", p["model_bytes_per_access"] if p["pattern"] == "scatter" else "")
    if "--write" in sys.argv:
        with open(os.path.join(ROOT, "profiles", "pmc_summary.json"), "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
