"""Counter comparison of two builds of the traversal kernel on one workload (round 6):
one process per (build, PMC pass); the workload's batch traced back-to-back under a fixed launch
config so both builds run the same schedule. Under rocprofv3 --pmc:
  MRT_LIB_DIR=<lib dir> python tools/codegen_pmc.py [workload] [launches] [config json | {"saved": 1}]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-ray-tracing_amd"))
sys.path.insert(0, REPO)


def main():
    import torch
    import bench
    from mrt.tracer import Tracer
    wl = sys.argv[1] if len(sys.argv) > 1 else "bunny-primary-1024x768"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    cfg = json.loads(sys.argv[3]) if len(sys.argv) > 3 else {"saved": 1}
    if cfg.get("saved"):   # the package's saved schedules, locked at bind (as bench.py runs)
        from mrt.schedules import DEFAULT_PATH, ScheduleStore
        bench.STORE = ScheduleStore(DEFAULT_PATH)
    torch.cuda.set_device(0)
    scenes = bench.SceneCache(1, 0, "/tmp/mrt_bvhcache")
    e = scenes.get(bench.workload_spec(wl)[0])
    tr = Tracer(0)
    b = bench.Batches(wl, e["scene"], e["gbvh"], tr)   # binds the BVH (no saved schedules: bench.STORE unset)
    if not cfg.get("saved"):
        tr.set_config(autotune=0, **cfg)
    gos = [tr.launcher(rb, exact_rcp=True) for rb, _ in b.batches]
    for _ in range(n):
        for go in gos:
            go()
    torch.cuda.synchronize()
    a_, z_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a_.record()
    for _ in range(50):
        for go in gos:
            go()
    z_.record()
    torch.cuda.synchronize()
    tr.trace_batch(b.batches[-1][0], exact_rcp=True)   # the schedule the launches ran (last_info)
    print(json.dumps({"lib": os.environ.get("MRT_LIB_DIR", "lib"), "workload": wl, "config": cfg,
                      "locked": b.locked_from_store, "candidate": tr.last_info.get("autotune_candidate"),
                      "ms_per_launch": a_.elapsed_time(z_) / 50 / len(gos)}), flush=True)


def summary(src):
    """Per-launch means of every counter of the trace kernel's dispatches at the most frequent grid
    size, per (workload, build) directory prefix `<workload>_<build>_p<pass>`, as one table."""
    import collections
    import csv
    import glob
    table = collections.defaultdict(dict)
    for d in sorted(glob.glob(f"{src}/*_p[0-9]")):
        key = os.path.basename(d).rsplit("_p", 1)[0]
        rows = []
        for f in glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True):
            rows += [r for r in csv.DictReader(open(f)) if "trace_kernel" in r["Kernel_Name"]]
        grid = lambda r: (r["Kernel_Name"], int(r.get("Grid_Size") or r.get("Grid_Size_X")))
        top = collections.Counter(grid(r) for r in rows).most_common(1)
        if not top:
            continue
        vals = collections.defaultdict(list)
        for r in rows:
            if grid(r) == top[0][0]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        table[key].update({k: sum(v) / len(v) for k, v in vals.items()})
    keys = sorted(table)
    names = sorted({n for k in keys for n in table[k]})
    wd = max(len(k) for k in keys) + 2
    print("%-26s" % "counter" + "".join("%*s" % (wd, k) for k in keys))
    for n in names:
        print("%-26s" % n + "".join("%*.0f" % (wd, table[k].get(n, float("nan"))) for k in keys))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        main()
