"""tools/prof_window.py keeps exactly the dispatches enqueued between the bench's marker
kernels (k_mark<1>/<2>: the timed batches; k_mark<3>/<4>: their serial replay), so a
kernel's rocprof average can be compared with the bench line's HIP-event timing."""
import csv
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("prof_window", os.path.join(ROOT, "tools", "prof_window.py"))
pw = importlib.util.module_from_spec(spec)
spec.loader.exec_module(pw)

FIELDS = ["Kind", "Agent_Id", "Queue_Id", "Stream_Id", "Thread_Id", "Dispatch_Id", "Kernel_Id", "Kernel_Name",
          "Correlation_Id", "Start_Timestamp", "End_Timestamp"]


def _trace(tmp_path, rows):
    p = tmp_path / "run_kernel_trace.csv"
    with open(p, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=FIELDS)
        w.writeheader()
        t = 0
        for i, (name, dur_us) in enumerate(rows):
            w.writerow({"Kind": "KERNEL_DISPATCH", "Dispatch_Id": i + 1, "Kernel_Name": name,
                        "Start_Timestamp": t, "End_Timestamp": t + int(dur_us * 1000)})
            t += int(dur_us * 1000) + 500
    return str(p)


def test_windows(tmp_path):
    fold = "void (anonymous namespace)::k_fold_wide<true>(unsigned int const*, int)"
    rows = [(fold, 27000.0),                                   # warm-up: outside every window
            ("void (anonymous namespace)::k_mark<1>(unsigned int*)", 1.0),
            (fold, 900.0), ("(anonymous namespace)::k_hist_dig(unsigned char const*)", 60.0), (fold, 1000.0),
            ("void (anonymous namespace)::k_mark<2>(unsigned int*)", 1.0),
            ("void (anonymous namespace)::k_mark<3>(unsigned int*)", 1.0),
            (fold, 800.0), (fold, 810.0),
            ("void (anonymous namespace)::k_mark<4>(unsigned int*)", 1.0),
            (fold, 5000.0)]                                    # after the replay: outside
    w = pw.windows(_trace(tmp_path, rows))
    assert w["timed"]["k_fold_wide<true>"]["calls"] == 2
    assert w["timed"]["k_fold_wide<true>"]["avg_us"] == 950.0
    assert w["timed"]["k_hist_dig"]["calls"] == 1
    assert w["replay"]["k_fold_wide<true>"] == {"calls": 2, "avg_us": 805.0, "min_us": 800.0, "max_us": 810.0,
                                                "total_us": 1610.0}
    assert all("k_mark" not in k for k in w["timed"]) and all("k_mark" not in k for k in w["replay"])


def test_missing_markers(tmp_path):
    w = pw.windows(_trace(tmp_path, [("void (anonymous namespace)::k_fold_wide<true>(int)", 1.0)]))
    assert w == {}
