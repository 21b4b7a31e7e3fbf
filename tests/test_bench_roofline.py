"""bench.py's roofline, on the CPU. The contract's fields: achieved = the SURVEY §8(d)
algorithmic bytes per launch / kernel time against the 8 TB/s HBM peak (cache-resident
scenes may pass 1, stated), traffic = the PMC fabric bytes per launch of a committed
profile (tools/summarize_prof.py) of the SAME schedule; beside them, what each level
served priced against its own ceiling (`served`, `binding_level`)."""
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
        with open(tmp_path / "profiles" / f"{bench.PROFILE_TAGS[0]}_{name}{rcp}_pmc_summary.json", "w") as f:
            json.dump(doc, f)
    return write


def test_contract_fields_and_served_levels(profile):
    profile("w", l2=2.0e9, fabric=0.3e9, avg_ns=100_000)
    r = bench.roofline("w", 6.0e9, 0.1, 10 << 20, SCHED)   # 6 GB of algorithmic bytes in 0.1 ms: 60 TB/s
    assert r["bound"] == "l2" and r["unit"] == "GB/s" and r["peak"] == bench.HBM_PEAK_GBS   # L2 serves 58 %
    assert r["achieved"] == pytest.approx(60000.0)
    assert r["frac"] == pytest.approx(60000.0 / bench.HBM_PEAK_GBS, rel=1e-3) and r["frac"] > 1.0
    assert "cache-resident" in r["note"]   # stated, not clamped
    assert r["served"]["l2"]["GBps"] == pytest.approx(20000.0)
    assert r["served"]["fabric"]["GBps"] == pytest.approx(3000.0)
    assert r["binding_level"] == "l2"
    assert r["traffic"] == int(0.3e9)
    assert r["hbm_measured_frac"] == pytest.approx(3000.0 / bench.HBM_PEAK_GBS, rel=1e-3)
    assert r["profile"]["kernel_ms_ratio"] == pytest.approx(1.0)


def test_fabric_binding(profile):
    profile("w", l2=1.0e9, fabric=0.7e9, avg_ns=100_000)
    r = bench.roofline("w", 2.0e9, 0.1, 900 << 20, SCHED)
    assert r["binding_level"] == "fabric" and r["bvh_exceeds_mall"] and r["bound"] == "hbm"   # 81 % of 8.6 TB/s
    assert r["frac"] == pytest.approx(20000.0 / bench.HBM_PEAK_GBS, rel=1e-3)


def test_profile_of_another_schedule_is_not_cited(profile):
    profile("w", l2=1.0e9, fabric=0.1e9, avg_ns=100_000, sched=dict(SCHED, autotune_candidate=0))
    r = bench.roofline("w", 2.0e9, 0.1, 10 << 20, SCHED)
    assert r["frac"] is not None and r["traffic"] is None and "no committed PMC profile" in r["profile"]["note"]


def test_newest_profile_of_the_schedule_is_cited(profile, tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "PROFILE_TAGS", ("new", "old"))
    for tag, fabric in (("new", 0.2e9), ("old", 0.1e9)):
        doc = {"avg_ns": 100_000, "schedule": SCHED, "l2_hit_rate": 0.5,
               "levels": {"l2_request_bytes": 1e9, "fabric_read_bytes": fabric, "write_bytes": 0, "fabric_bytes": fabric}}
        with open(tmp_path / "profiles" / f"{tag}_w_pmc_summary.json", "w") as f:
            json.dump(doc, f)
    assert bench.roofline("w", 2.0e9, 0.1, 10 << 20, SCHED)["traffic"] == int(0.2e9)


def test_missing_profile(profile):
    r = bench.roofline("nothing", 2.0e9, 0.1, 10 << 20, SCHED)
    assert r["traffic"] is None and "no committed PMC profile" in r["profile"]["note"]


def test_fast_rcp_profile_is_separate(profile):
    profile("w", l2=1.0e9, fabric=0.1e9, avg_ns=100_000, rcp="_rcpfast")
    assert bench.roofline("w", 2.0e9, 0.1, 10 << 20, SCHED)["traffic"] is None
    assert bench.roofline("w", 2.0e9, 0.1, 10 << 20, SCHED, rcp="fast")["traffic"] is not None


def test_schedule_names():
    assert bench.schedule_name(-1) == "fixed rule"
    assert bench.schedule_name(2) == bench.SCHEDULES[2]
    assert bench.schedule_name(8 | (3 << 8)).endswith("spec_slack 4")
    assert bench.schedule_name(10 | (0 << 8)).endswith("no frontier tail")


def test_latency_bound_when_every_level_is_lightly_served(profile):
    """the bound is read from the served fractions — a launch whose levels
    all serve under 25 % of their ceilings is latency-bound, not HBM-bound."""
    profile("w", l2=1.0e9, fabric=0.1e9, avg_ns=100_000)    # L2: 10 TB/s of 34.5 = 29 %
    r = bench.roofline("w", 2.0e9, 0.1, 10 << 20, SCHED)
    assert r["served"]["l2"]["frac"] > bench.LATENCY_BOUND and r["bound"] == "l2"
    profile("w", l2=0.5e9, fabric=0.1e9, avg_ns=100_000)    # 14 % of L2, 12 % of the fabric
    r = bench.roofline("w", 2.0e9, 0.1, 10 << 20, SCHED)
    assert max(v["frac"] for v in r["served"].values()) < bench.LATENCY_BOUND and r["bound"] == "latency"


def test_kernel_bytes_give_their_own_frac(profile):
    profile("w", l2=0.5e9, fabric=0.1e9, avg_ns=100_000)
    r = bench.roofline("w", 9.0e9, 0.1, 10 << 20, SCHED, kernel_bytes_per_launch=6.0e9)
    assert r["frac"] == pytest.approx(90000.0 / bench.HBM_PEAK_GBS, rel=1e-3)        # SURVEY 8(d), kept
    assert r["kernel_frac"] == pytest.approx(60000.0 / bench.HBM_PEAK_GBS, rel=1e-3)
    assert r["kernel_bytes_per_launch"] == int(6.0e9)


@pytest.mark.parametrize("avg_ns,cited", [(100_000, True), (108_000, True), (115_000, False), (62_500, False)])
def test_profile_at_another_speed_is_not_cited(profile, avg_ns, cited):
    """a profile of the same schedule whose mean kernel time is outside
    [0.9, 1.1] of this run's (the gloo rehearsal cited one at 0.625) is not cited."""
    profile("w", l2=1.0e9, fabric=0.1e9, avg_ns=avg_ns)
    r = bench.roofline("w", 2.0e9, 0.1, 10 << 20, SCHED)
    assert (r["traffic"] is not None) == cited
    if not cited:
        assert "not cited" in r["profile"]["note"] and r["profile"]["kernel_ms_ratio"] == pytest.approx(avg_ns / 1e5)
