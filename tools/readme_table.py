"""Every scene x ray-type cell of the reference's README performance table
(README.md:60-81) measured on one MI355X with bench.py's workload code, next to
the README's Kepler Mrays/s.

Same measurement as bench.py (exact-rcp production kernel, device-generated
rays, rays counted / kernel time of the timed steps); per cell also the
oracle's agreement on every ray of every batch of the cell (closest hit: id and
t bit-identical; any hit: "valid hits" — hit/miss identical and every hit that differs
from the oracle's re-verified as a Woop hit with exactly its t; `--parity-rays N` checks a prefix
of N rays per batch instead). Scenes are the
deterministic stand-ins of csrc/host/scene.cpp; fairy, sibenik and san have no
size in the README (their commonly distributed triangle counts are assumed).

  python tools/readme_table.py [--bvh-cache DIR] [--steps K] [--cells a,b,...]

Writes gpurun_out/readme_table.json and gpurun_out/readme_table.md.
"""
import argparse
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

# README rows in table order: (workload, README Mrays/s, README line).
CELLS = [
    ("sponza-primary-640x480", 597.51, 61), ("mori-primary-640x480", 1271.61, 62),
    ("hairball-primary-640x480", 280.49, 63), ("dragon-primary-640x480", 575.43, 64),
    ("bunny-primary-640x480", 825.11, 65),
    ("conference-diffuse-640x480", 831.28, 68), ("fairy-diffuse-640x480", 678.77, 69),
    ("sibenik-diffuse-640x480", 286.97, 70), ("san-diffuse-640x480", 132.28, 71),
    ("sponza-diffuse-640x480", 325.33, 72), ("mori-diffuse-640x480", 1466.05, 73),
    ("conference-ao-640x480", 1478.43, 76), ("fairy-ao-640x480", 1280.77, 77),
    ("sibenik-ao-640x480", 1499.86, 78), ("san-ao-640x480", 556.89, 79),
    ("sponza-ao-640x480", 1022.61, 80), ("mori-ao-640x480", 2763.01, 81),
]


def heartbeat(stop, state):
    # The GPU pool takes 3 silent minutes for a hang; the big SBVH builds are long and quiet.
    while not stop.wait(30):
        print(f"  ... {state['cell']} ({time.perf_counter() - state['t0']:.0f} s)", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bvh-cache", default="/tmp/mrt_bvhcache")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--parity-rays", type=int, default=0, help="rays per batch checked against the oracle (0 = all)")
    ap.add_argument("--cells", default="", help="comma-separated subset of workloads")
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out"))
    ap.add_argument("--cell-db", default=None,
                    help="tools/tune_db.py --out-cells file: each cell locks its own tuned schedule (after the BVH's "
                         "saved ones), so two ray types of one BVH and batch size each run their own")
    ap.add_argument("--tune-db", default=None,
                    help="saved schedules to lock (default: the package's; 'none': every cell's batch size is tuned "
                         "live in its warmup, so two ray types of one BVH and batch size never share a schedule)")
    args = ap.parse_args()

    import numpy as np
    import torch
    import bench
    import oracle_lib as O
    from mrt.tracer import Tracer

    from mrt.schedules import DEFAULT_PATH, ScheduleStore
    torch.cuda.set_device(0)
    tracer = Tracer(0)
    # cells without a saved schedule for their BVH and batch size autotune in the warmup
    bench.STORE = None if args.tune_db == "none" else ScheduleStore(args.tune_db or DEFAULT_PATH)
    cell_db = {}
    if args.cell_db:
        with open(args.cell_db) as f:
            cdb = json.load(f)
        from mrt import _lib
        if cdb.get("version") == _lib.MRT_TUNE_VERSION:
            cell_db = cdb["cells"]
    want = set(args.cells.split(",")) if args.cells else None
    state = {"cell": "start", "t0": time.perf_counter()}
    stop = threading.Event()
    threading.Thread(target=heartbeat, args=(stop, state), daemon=True).start()
    rows = []
    scenes = bench.SceneCache(1, 0, args.bvh_cache)
    for name, readme, line in CELLS:
        if want and name not in want:
            continue
        state.update(cell=name, t0=time.perf_counter())
        scene_name = bench.workload_spec(name)[0]
        e = scenes.get(scene_name)
        scene, build_s = e["scene"], e["build_s"]
        bufs = scenes.host_buffers(scene_name)
        batches = bench.Batches(name, scene, e["gbvh"], tracer)
        own = cell_db.get(name)
        if own and own["fingerprint"] == e["gbvh"].fingerprint:   # this cell's own tuned schedule
            from mrt import _lib
            tracer.load_schedules([(n, v, own["candidate"], _lib.MRT_TUNE_VERSION) for n, v in own["keys"]])
        alg_bytes, n_nodes, n_tris, n_leaves = bench.algorithmic_bytes(tracer, batches.batches)
        launches = [tracer.launcher(rb, exact_rcp=True) for rb, _ in batches.batches]
        wall, launch_ms, _ = bench.time_steps(launches, args.steps, args.warmup, 1)
        value = batches.rays_counted * args.steps / wall / 1e6
        kernel_ms = launch_ms * len(batches.batches)
        # Parity of every ray of every batch (the timed launches' results) against the oracle.
        n, same, checked, ties = 0, 0, 0, 0
        for rb, _ in batches.batches:
            k = rb.size if args.parity_rays <= 0 else min(args.parity_rays, rb.size)
            rays = rb.rays.cpu().numpy()[:k]
            gpu = rb.results_numpy()[:k]
            any_hit = not rb.need_closest_hit
            ref, _, _ = O.trace(rays, *bufs, any_hit=any_hit, threads=bench.host_threads())
            if any_hit:   # hit/miss identical, and every differing hit re-verified as a Woop hit with its t
                ok = (gpu[:, 0] == -1) == (ref[:, 0] == -1)
                diff = np.nonzero((gpu[:, 0] != ref[:, 0]) | (gpu[:, 1] != ref[:, 1]))[0]
                ok[O.invalid_hits(rays, gpu, bufs[1], bufs[2], which=diff)] = False
                same += int(ok.sum())
                checked += len(diff)
            else:
                eq = (gpu[:, 0] == ref[:, 0]) & (gpu[:, 1] == ref[:, 1])
                same += int(eq.sum())
                # another triangle at exactly the oracle's t (coincident surfaces): which one wins follows
                # the traversal order; counted apart, each re-verified as a Woop hit at that t
                t_eq = np.nonzero(~eq & (gpu[:, 1] == ref[:, 1]))[0]
                ties += len(t_eq) - len(O.invalid_hits(rays, gpu, bufs[1], bufs[2], which=t_eq))
            n += k
        agree = same / max(1, n)
        row = {
            "workload": name, "readme_mrays": readme, "readme_line": line,
            "mrays": round(value, 2), "x_readme": round(value / readme, 2),
            "kernel_ms": round(kernel_ms, 4), "rays_counted": batches.rays_counted, "rays_traced": batches.rays_traced,
            "tris": scene.num_triangles, "inner_nodes": len(bufs[0]) // 16,
            "bvh_mb": round(4 * (len(bufs[0]) + len(bufs[1]) + len(bufs[2])) / 2**20, 1), "build_s": round(build_s, 1),
            "per_ray": {"nodes": round(n_nodes / batches.rays_traced, 2), "tris": round(n_tris / batches.rays_traced, 2)},
            "alg_gbs": round(alg_bytes / (kernel_ms * 1e-3) / 1e9, 1),
            "schedule": bench.schedule_of(tracer, batches.batches[0][0], True)["name"],
            # the saved schedules the cell ran (checked against the shipped table by
            # tests/test_readme_table.py): the BVH's fingerprint and its entries for the cell's batch sizes
            "fingerprint": e["gbvh"].fingerprint,
            "schedules": sorted({tuple(x[:3]) for x in tracer.schedules()
                                 if x[0] in {rb.size for rb, _ in batches.batches}}),
            "parity_rays": n, "parity_all_rays": n == batches.rays_traced, "parity_agree": agree, "parity_kind": "valid hits" if any_hit else "id+t exact",
            "any_hit_results_reverified": checked if any_hit else None,
            "parity_same": same, "exact_t_ties": None if any_hit else ties,
        }
        rows.append(row)
        print(json.dumps(row), flush=True)
        del batches, bufs, scene, launches
        scenes.entries.pop(scene_name, None)
        torch.cuda.empty_cache()
    stop.set()

    os.makedirs(args.out, exist_ok=True)
    with open(os.path.join(args.out, "readme_table.json"), "w") as f:
        json.dump(rows, f, indent=1)
    write_md(rows, args.out)


# README.md:48-58: the reference scenes' inner-node counts (its SBVH on the real assets; the stand-ins here
# have the same triangle counts but other geometry, so their counts are a plausibility check only)
README_INNER_NODES = {"bunny": 50876, "dragon": 301376, "conference": 105025, "hairball": 1249052, "sponza": 35907,
                      "mori": 3483}


def agreement(r):
    """The oracle column: counts, not a rounded fraction (5 ties in 307 200 rays read 1.0000)."""
    n = r["parity_rays"]
    if r.get("parity_same") is None:   # a row of an older run
        return f"{r['parity_agree']:.6f} ({r['parity_kind']}, {n} rays)"
    same = r["parity_same"]
    if r["parity_kind"] == "valid hits":
        return f"{same}/{n} valid hits ({r['any_hit_results_reverified']} differing hits re-verified)"
    ties = r.get("exact_t_ties") or 0
    other = n - same - ties
    text = f"{same}/{n} id+t exact"
    if ties:
        text += f", {ties} exact-t ties (another triangle at the oracle's t, a valid hit)"
    if other:
        text += f", **{other} other**"
    return text


def write_md(rows, out):
    # alg. GB/s: SURVEY §8(d)'s bytes per ray (cache hits included) over the kernel time; a rate, not a level's
    # traffic, so it may exceed the HBM peak (bench.py's roofline prices the per-level PMC bytes instead)
    md = ["| README cell | tris (stand-in) | inner nodes (stand-in / README) | README Mrays/s | MI355X Mrays/s | "
          "× README | kernel ms | nodes/ray | tris/ray | alg. GB/s (not a roofline) | schedule | oracle agreement |",
          "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        ref = README_INNER_NODES.get(r["workload"].split("-")[0])
        nodes = f"{r['inner_nodes']:,} / {ref:,}" if ref else f"{r['inner_nodes']:,} / —"
        md.append(f"| {r['workload']} (README:{r['readme_line']}) | {r['tris']:,} | {nodes} | {r['readme_mrays']} | "
                  f"**{r['mrays']}** | {r['x_readme']} | {r['kernel_ms']} | {r['per_ray']['nodes']} | "
                  f"{r['per_ray']['tris']} | {r['alg_gbs']} | {r.get('schedule', '')} | {agreement(r)} |")
    with open(os.path.join(out, "readme_table.md"), "w") as f:
        f.write("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    if len(sys.argv) == 3 and sys.argv[1] == "--md-from":   # re-render the table from a saved JSON
        write_md(json.load(open(sys.argv[2])), os.path.dirname(os.path.abspath(sys.argv[2])))
    else:
        main()
