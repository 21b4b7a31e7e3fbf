"""tools/readme_table.py's oracle column (CPU only): counts instead of a rounded fraction, exact-t ties
apart from other mismatches, and the committed round-5 table is consistent with its JSON rows (every cell
checked on all of its rays; the only closest-hit differences are San Miguel diffuse's exact-t ties)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import readme_table as rt  # noqa: E402


def row(**kw):
    r = {"parity_rays": 307200, "parity_kind": "id+t exact", "parity_agree": 1.0, "parity_same": 307200,
         "exact_t_ties": 0, "any_hit_results_reverified": None}
    r.update(kw)
    return r


def test_agreement_counts_ties_apart():
    assert rt.agreement(row()) == "307200/307200 id+t exact"
    t = rt.agreement(row(parity_same=307195, exact_t_ties=5))
    assert t.startswith("307195/307200 id+t exact, 5 exact-t ties") and "other**" not in t
    t = rt.agreement(row(parity_same=307190, exact_t_ties=5))
    assert t.endswith("**5 other**")
    t = rt.agreement(row(parity_kind="valid hits", any_hit_results_reverified=791, exact_t_ties=None))
    assert t == "307200/307200 valid hits (791 differing hits re-verified)"


def test_agreement_of_an_older_row_keeps_six_digits():
    r = row(parity_agree=0.9999837239583333)
    del r["parity_same"]
    assert rt.agreement(r).startswith("0.999984")


def test_committed_round5_table_is_complete():
    with open(os.path.join(REPO, "profiles", "round5_readme_table.json")) as f:
        rows = json.load(f)
    assert {r["workload"] for r in rows} == {c[0] for c in rt.CELLS}
    for r in rows:
        assert r["parity_all_rays"] and r["parity_rays"] == r["rays_traced"]
        assert r["x_readme"] > 1
        if r["parity_kind"] == "valid hits":
            assert r["parity_same"] == r["parity_rays"]
        else:
            assert r["parity_same"] + r["exact_t_ties"] == r["parity_rays"]
            if r["workload"] != "san-diffuse-640x480":
                assert r["exact_t_ties"] == 0


def test_committed_round6_table_runs_the_shipped_schedules():
    """the README table must report what a user of the shipped schedule table
    gets — every row's saved schedules (fingerprint, batch size, variant -> candidate) equal the
    package's mrt/tuned_schedules.json entries, so no cell depends on a per-cell lock."""
    import pytest
    path = os.path.join(REPO, "profiles", "round6_readme_table.json")
    if not os.path.exists(path):
        pytest.skip("no round-6 table")
    with open(path) as f:
        rows = json.load(f)
    with open(os.path.join(REPO, "gpu-ray-tracing_amd", "mrt", "tuned_schedules.json")) as f:
        shipped = json.load(f)
    assert {r["workload"] for r in rows} == {c[0] for c in rt.CELLS}
    for r in rows:
        table = {(n, v): c for n, v, c, _ in shipped["bvhs"][r["fingerprint"]]}
        assert r["schedules"], r["workload"]
        for n, v, c in r["schedules"]:
            assert table.get((n, v)) == c, (r["workload"], n, v, c, table.get((n, v)))
        assert r["x_readme"] > 1 and r["parity_all_rays"]
