"""Condense a tools/profile_round.sh output directory into profiles/<tag>_*:
the rocprofv3 kernel-stats CSV as-is, and a JSON with the per-launch PMC
values of the timed trace kernel (FETCH_SIZE / WRITE_SIZE in KB as rocprofv3
reports them, gfx950 read correction per MI355X_MICROARCH.md §HBM)."""
import collections
import csv
import json
import os
import shutil
import sys

src, tag = sys.argv[1], sys.argv[2]
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(repo, "profiles")
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))

# the timed kernel = the trace_kernel instantiation with the most calls
stats = list(csv.DictReader(open(os.path.join(src, "kt", "run_kernel_stats.csv"))))
timed = max((r for r in stats if "trace_kernel" in r["Name"]), key=lambda r: int(r["Calls"]))
out = {"kernel": timed["Name"], "calls": int(timed["Calls"]), "avg_ns": float(timed["AverageNs"]),
       "min_ns": float(timed["MinNs"]), "max_ns": float(timed["MaxNs"]), "pmc": {}}
for p in sorted(d for d in os.listdir(src) if d.startswith("pmc")):
    rows = list(csv.DictReader(open(os.path.join(src, p, "run_counter_collection.csv"))))
    vals = collections.defaultdict(list)
    grid = {}
    for r in rows:
        if r["Kernel_Name"] == timed["Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            grid = {"grid_size": int(r["Grid_Size"]), "rocprof_VGPR_Count_field": int(r["VGPR_Count"]), "lds": int(r["LDS_Block_Size"])}
    for k, v in vals.items():
        out["pmc"][k] = {"per_launch_mean": sum(v) / len(v), "launches": len(v)}
    out.update(grid)
pm = out["pmc"]
if "FETCH_SIZE" in pm and "WRITE_SIZE" in pm:
    fetch = pm["FETCH_SIZE"]["per_launch_mean"] * 1024
    write = pm["WRITE_SIZE"]["per_launch_mean"] * 1024
    out["hbm_bytes_per_launch"] = {"fetch_raw": fetch, "fetch_corrected_x2": 2 * fetch, "write": write,
                                   "total_corrected": 2 * fetch + write,
                                   "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 reports 1/2 of "
                                           "wide reads); our 16-B-per-lane gathers are not a calibrated width"}
if "TCC_HIT_sum" in pm and "TCC_MISS_sum" in pm:
    h, m = pm["TCC_HIT_sum"]["per_launch_mean"], pm["TCC_MISS_sum"]["per_launch_mean"]
    out["l2_hit_rate"] = h / (h + m)
json.dump(out, open(os.path.join(dst, f"{tag}_pmc_summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
