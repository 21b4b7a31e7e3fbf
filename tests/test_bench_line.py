"""bench.py's stdout line stays parseable (the driver did not parse round 3's
21.7 kB line): built by bench.make_line from recorded runs — round 3's full line converted
to the detail structure, and the committed round-4 detail file when present — it is one
JSON object under bench.LINE_MAX_BYTES with the contract's fields, at N = 1 (weak: the
headline) and N > 1 (strong: the sharded hairball RayBuffer)."""
import argparse
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def args_for(scaling, workload=bench.HEADLINE):
    return argparse.Namespace(workload=workload, scaling=scaling, steps=200, warmup=20, strong_steps=10, rcp="exact")


def round3_detail():
    """profiles/round3_bench_n1.json (the line the driver could not parse) as head/extras/strong."""
    with open(os.path.join(REPO, "profiles", "round3_bench_n1.json")) as f:
        d = json.load(f)
    head = dict(d["detail"])
    head.update({"workload": d["config"]["workload"], "value": d["value"], "ms_per_step": d["ms_per_step"],
                 "scene_tris": d["config"]["scene_tris"], "rays_counted": d["config"]["rays_per_gpu"],
                 "roofline": d["roofline"], "cpu_baseline": d["cpu_baseline"], "rcp_fast": d["rcp_fast"]})
    return head, d["extra_workloads"], d["strong_scaling"]


def details():
    out = [("round3", *round3_detail(), None)]
    for tag in ("round4", "round5"):
        path = os.path.join(REPO, "profiles", f"{tag}_bench_detail.json")
        if os.path.exists(path):
            with open(path) as f:
                d = json.load(f)
            out.append((tag, d["head"], d["extras"], d["strong"], d.get("readme_cells")))
    return out


@pytest.mark.parametrize("rec", details(), ids=lambda r: r[0])
def test_line_is_small_and_complete_at_n1(rec):
    _, head, extras, strong, cells = rec
    line, detail = bench.make_line(args_for("weak"), 1, head, extras, strong, {}, cells)
    text = json.dumps(line, separators=(",", ":"))
    assert len(text) < 10_000 and len(text) <= bench.LINE_MAX_BYTES
    assert "\n" not in text and json.loads(text) == line
    for k in CONTRACT:
        assert k in line, k
    assert line["scaling"] == "weak" and line["value"] == head["value"]
    rf = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    assert line["cpu_baseline"]["value"] > 0 and line["cpu_baseline"]["cores"] >= 1
    assert len(line["extra_workloads"]) == len(extras)
    for e in line["extra_workloads"]:
        assert e["value"] > 0 and "parity" in e and "roofline" in e
    sp = line["strong_scaling"]
    assert "shard_ms" not in json.dumps(sp) and sp["projected_from_one_gpu"]["8"]["eta"] > 0
    # everything dropped from the line stays in the detail
    assert detail["head"] is head and detail["extras"] is extras and detail["strong"] is strong


@pytest.mark.parametrize("rec", details(), ids=lambda r: r[0])
def test_line_at_n_gt_1_is_the_strong_scaling_number(rec):
    """at N > 1 the value is the sharded hairball RayBuffer (BASELINE configs[4]),
    ms_per_step its T_n, the parallelism names block-cyclic shards; weak scaling is a sub-block."""
    _, head, _, strong, _ = rec
    st = dict(strong, n_gpus=2, tn_ms=strong["t1_ms"] / 1.9, eta=0.95)
    st["value"] = round(st["rays_counted"] / (st["tn_ms"] * 1e-3) / 1e6, 2)
    line, _ = bench.make_line(args_for("strong"), 2, head, [], st, {})
    assert line["value"] == st["value"] and line["ms_per_step"] == st["tn_ms"] and line["scaling"] == "strong"
    assert line["config"]["workload"] == bench.STRONG["name"]
    assert "block-cyclic" in line["config"]["parallelism"] and "contiguous" not in line["config"]["parallelism"]
    assert line["weak_scaling"]["value"] == head["value"]
    assert line["strong_scaling"]["value_n1_same_run"] > 0
    assert len(json.dumps(line)) < 10_000


def test_readme_cells_ride_on_the_n1_line():
    """The README cells of a default N = 1 run (bench.README_N1) are on the line, each with its ratio to the
    README and the oracle agreement, and the line with all of them still fits (the newest recorded run)."""
    paths = [os.path.join(REPO, "profiles", f"round{r}_bench_detail.json") for r in (6, 5)]
    paths = [p for p in paths if os.path.exists(p)]
    if not paths:
        pytest.skip("no recorded detail file")
    path = paths[0]
    with open(path) as f:
        d = json.load(f)
    cells = d.get("readme_cells")
    if not cells:
        pytest.skip("recorded run without README cells")
    line, _ = bench.make_line(args_for("weak"), 1, d["head"], d["extras"], d["strong"], {}, cells)
    text = json.dumps(line, separators=(",", ":"))
    assert len(text) <= bench.LINE_MAX_BYTES
    got = {c["cell"] for c in line["readme_cells"]}
    assert got == {c["cell"] for c in cells} and got <= set(bench.README_N1)
    if "round6" in path:
        assert got == set(bench.README_N1)   # round 6: all 17 README cells, San Miguel included
    for c in line["readme_cells"]:
        # closest hits: every ray equal, or the rest exact-t ties (another valid triangle at the oracle's t)
        assert c["x_readme"] > 1 and (c["agree"] == 1.0 or c.get("ties", 0) > 0)
        assert abs(c["value"] / bench.REFERENCE_MRAYS[c["cell"]] - c["x_readme"]) < 0.01
