"""Summary of one tools/pmc_configs.sh pass: per-launch means of the counters over the trace
kernel's dispatches at the most frequent grid size (the timed launches), as bytes:
  l2_req  = TCP_TCC_READ_REQ x 128 B   (lines the L1s fetched from L2)
  fabric  = TCC_EA0_RDREQ x 128 B      (lines L2 fetched from the Infinity Cache / HBM)
(gfx950 line size, profiles/round3_counter_calibration.md). Usage: pmc_configs.py DIR CONFIG MS"""
import collections
import csv
import glob
import json
import sys

src, cfg, ms = sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else ""
rows = []
for f in glob.glob(f"{src}/**/run_counter_collection.csv", recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if "trace_kernel" in r["Kernel_Name"]]
grid = lambda r: int(r.get("Grid_Size") or r.get("Grid_Size_X"))
by = collections.Counter((r["Kernel_Name"], grid(r)) for r in rows if r["Counter_Name"] == "TCC_HIT_sum")
(kname, g), n = by.most_common(1)[0]
vals = collections.defaultdict(list)
for r in rows:
    if r["Kernel_Name"] == kname and grid(r) == g:
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in vals.items()}
hit = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
print(json.dumps({"config": json.loads(cfg), "kernel_ms": ms, "launches": n, "grid_lanes": g,
                  "l2_req_MB": round(m["TCP_TCC_READ_REQ_sum"] * 128 / 1e6, 1),
                  "fabric_MB": round(m["TCC_EA0_RDREQ_sum"] * 128 / 1e6, 1), "l2_hit": round(hit, 4)}), flush=True)
