"""bench.py's per-level roofline, on the CPU: the bytes each cache
level served (from a PMC summary written by tools/summarize_prof.py) priced against
that level's ceiling; the binding level's fraction is the line's `frac`; a profile
whose schedule differs from the timed one is not cited."""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

SCHED = {"autotune_candidate": 2, "grid_waves": 2048, "num_queues": 8, "fetch_threshold": 0}


@pytest.fixture
def profile(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    os.makedirs(tmp_path / "profiles")

    def write(name, l2, fabric, avg_ns, sched=SCHED, rcp=""):
        doc = {"avg_ns": avg_ns, "schedule": sched, "l2_hit_rate": 0.5,
               "levels": {"l2_request_bytes": l2, "fabric_read_bytes": fabric, "write_bytes": 0,
                          "fabric_bytes": fabric}}
        with open(tmp_path / "profiles" / f"{bench.PROFILE_TAG}_{name}{rcp}_pmc_summary.json", "w") as f:
            json.dump(doc, f)
    return write


def test_binding_level_and_bounded_fraction(profile):
    profile("w", l2=2.0e9, fabric=0.3e9, avg_ns=100_000)
    r = bench.roofline("w", 6.0e9, 0.1, 10 << 20, SCHED)   # 6 GB of algorithmic bytes in 0.1 ms: 60 TB/s
    assert r["algorithmic"]["GBps"] == pytest.approx(60000.0)
    assert r["levels"]["l2"]["GBps"] == pytest.approx(20000.0)
    assert r["levels"]["fabric"]["GBps"] == pytest.approx(3000.0)
    assert r["bound"] == "l2" and r["peak"] == bench.L2_PEAK_GBS
    assert r["frac"] == pytest.approx(20000.0 / bench.L2_PEAK_GBS, rel=1e-3) and r["frac"] <= 1.0
    assert r["traffic"] == int(0.3e9)
    assert r["hbm_measured_frac"] == pytest.approx(3000.0 / bench.HBM_PEAK_GBS, rel=1e-3)
    assert r["profile"]["kernel_ms_ratio"] == pytest.approx(1.0)


def test_fabric_bound(profile):
    profile("w", l2=1.0e9, fabric=0.7e9, avg_ns=100_000)
    r = bench.roofline("w", 2.0e9, 0.1, 900 << 20, SCHED)
    assert r["bound"] == "fabric" and r["peak"] == bench.MALL_PEAK_GBS and r["bvh_exceeds_mall"]


def test_profile_of_another_schedule_is_not_cited(profile):
    profile("w", l2=1.0e9, fabric=0.1e9, avg_ns=100_000, sched=dict(SCHED, autotune_candidate=0))
    r = bench.roofline("w", 2.0e9, 0.1, 10 << 20, SCHED)
    assert r["frac"] is None and r["traffic"] is None and "differs" in r["note"]


def test_missing_profile(profile):
    r = bench.roofline("nothing", 2.0e9, 0.1, 10 << 20, SCHED)
    assert r["frac"] is None and "no committed PMC profile" in r["note"]


def test_fast_rcp_profile_is_separate(profile):
    profile("w", l2=1.0e9, fabric=0.1e9, avg_ns=100_000, rcp="_rcpfast")
    assert bench.roofline("w", 2.0e9, 0.1, 10 << 20, SCHED)["frac"] is None
    assert bench.roofline("w", 2.0e9, 0.1, 10 << 20, SCHED, rcp="fast")["frac"] is not None


def test_schedule_names():
    assert bench.schedule_name(-1) == "fixed rule"
    assert bench.schedule_name(2) == bench.SCHEDULES[2]
    assert bench.schedule_name(8 | (3 << 8)).endswith("spec_slack 4")
    assert bench.schedule_name(10 | (0 << 8)).endswith("no frontier tail")
