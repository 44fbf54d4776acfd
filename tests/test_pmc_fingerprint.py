"""The PMC bytes a bench line carries (roofline.traffic / step_traffic) must describe that
run: profiles/pmc_summary.json records the fingerprint of the bench run its rocprofv3
passes measured, and bench.py attaches the bytes only to a run with the same fingerprint,
otherwise null with a reason."""
import argparse
import json

import bench
import bench_kinds as bk


def _args(**kw):
    a = dict(workload="uniform", batch=1 << 26, steps=20, warmup=5, token_limit=10, tokens_per_period=1,
             period_ticks=10_000_000, interval_us=10_000, queue_limit=16, route="pre", share_device=False)
    a.update(kw)
    return argparse.Namespace(**a)


LAYOUT = {"passes": 2, "r_bits": 11, "packed": True, "hot": True, "pipeline": True, "narrow": True,
          "medium": False}


def _summary(tmp_path, fp):
    w = {"step_hbm_bytes": 9.19e9, "stages": {"fold": {"hbm_bytes_per_step": 3.39e9}},
         "kernels": {"k_fold_q<true>": {"hbm_bytes_per_launch": 6.5e9}}}
    if fp is not None:
        w["fingerprint"] = fp
    p = tmp_path / "pmc_summary.json"
    p.write_text(json.dumps({"workloads": {fp["workload"] if fp else "uniform": w}}))
    return str(p)


def test_matching_run_gets_the_bytes(tmp_path):
    fp = bk.run_fingerprint(_args(), 1, 100_000_000, LAYOUT)
    assert len(fp["engine_sources_sha256"]) == 64
    w, why = bk.pmc_workload("uniform", json.loads(json.dumps(fp)), _summary(tmp_path, fp))
    assert why is None and bench.pmc_stage(w, "fold") == 3.39e9 and bench.pmc_step_traffic(w) == 9.19e9


def test_mismatched_run_gets_null_and_a_reason(tmp_path):
    fp = bk.run_fingerprint(_args(), 1, 100_000_000, LAYOUT)
    path = _summary(tmp_path, fp)
    # the 2-rank rehearsal line of round 3: 50.5M keys per rank, world 2, share-device
    other = bk.run_fingerprint(_args(share_device=True), 2, 50_500_000, LAYOUT)
    w, why = bk.pmc_workload("uniform", other, path)
    assert w is None and "keys_per_gpu" in why and "world" in why
    assert bench.pmc_stage(w, "fold") is None and bench.pmc_step_traffic(w) is None
    # a different schedule, batch or layout each suffice
    for fp2 in (bk.run_fingerprint(_args(steps=10), 1, 100_000_000, LAYOUT),
                bk.run_fingerprint(_args(batch=1 << 20), 1, 100_000_000, LAYOUT),
                bk.run_fingerprint(_args(), 1, 100_000_000, dict(LAYOUT, narrow=False))):
        w, why = bk.pmc_workload("uniform", fp2, path)
        assert w is None and why.startswith("PMC passes ran a different configuration")
    # changed engine sources
    w, why = bk.pmc_workload("uniform", dict(fp, engine_sources_sha256="0" * 64), path)
    assert w is None and "engine_sources_sha256" in why


def test_summary_without_fingerprint_or_workload(tmp_path):
    fp = bk.run_fingerprint(_args(), 1, 100_000_000, LAYOUT)
    path = _summary(tmp_path, None)
    assert bk.pmc_workload("uniform", fp, path) == (None, "the PMC passes recorded no run fingerprint")
    w, why = bk.pmc_workload("zipf", fp, path)
    assert w is None and "zipf" in why
    w, why = bk.pmc_workload("uniform", fp, str(tmp_path / "absent.json"))
    assert w is None and why.startswith("no PMC summary")


def test_queue_roofline_traffic_follows_the_match(tmp_path, monkeypatch):
    fp = bk.run_fingerprint(_args(workload="queue", token_limit=4, interval_us=1000), 1, 100_000_000, LAYOUT)
    monkeypatch.setattr(bk, "PMC_SUMMARY", _summary(tmp_path, fp))
    monkeypatch.setattr(bk.pmc_workload, "__defaults__", (bk.PMC_SUMMARY,))
    stages = {"fold": 57.8, "scatter": 20.0}
    r = bk._roofline(2.89, 2.88e9, "B_alg", 3.84e9, "own", "queue", fp, 4.2, stages, 20)
    assert r["traffic"] == 6.5e9 and "traffic_null_reason" not in r
    # frac = the step's B_alg over the fold's launch time; the fold's own
    # bytes are reported beside it
    assert r["kernel"] == "fold" and r["frac"] == round(2.88e9 / 2.89e-3 / 1e9 / bk.HBM_PEAK_GBS, 4)
    assert r["kernel_own_bytes"] == int(3.84e9) and r["largest_stage"] == "fold"
    r = bk._roofline(2.89, 2.88e9, "B_alg", 3.84e9, "own", "queue", dict(fp, keys_per_gpu=12_500_000), 4.2,
                     stages, 20)
    assert r["traffic"] is None and "keys_per_gpu" in r["traffic_null_reason"]


def test_fold_kernel_names_cover_template_arguments():
    """k_fold_q carries its queue-header width as a template argument (round 6): the PMC
    entry "k_fold_q<true, unsigned int>" is the fold that PMC_KERNELS names "k_fold_q<true>"."""
    w = {"kernels": {"k_fold_q<true, unsigned int>": {"hbm_bytes_per_launch": 5.5e9},
                     "k_scatter_rec<true, false, true, false, false>": {"hbm_bytes_per_launch": 1.0}}}
    assert bk._pmc_traffic(w, bk.PMC_KERNELS[("queue", "fold")]) == 5.5e9
    assert bk._pmc_traffic({"kernels": {"k_fold_q<true>": {"hbm_bytes_per_launch": 6.0}}}, ["k_fold_q<true>"]) == 6.0
    assert bk._pmc_traffic({"kernels": {}}, ["k_fold_q<true>"]) is None
