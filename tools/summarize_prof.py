"""Condense a tools/profile_round.sh output directory into profiles/<tag>_*: the
rocprofv3 kernel-stats CSV as-is, and a JSON with the per-launch PMC values of the
timed trace kernel and the bytes each cache level served (bench.py roofline()):
  l2_request_bytes = TCP_TCC_READ_REQ x 128     (lines the L1s fetched from L2)
  fabric_bytes     = TCC_EA0_RDREQ x 128 (32-B requests x 32) + WRITE_SIZE
                     (L2 misses served by the Infinity Cache or HBM, and writes)
128 B per request: gfx950's line, calibrated by tools/ubench_levels.hip
(profiles/round3_counter_calibration.md). The schedule the profiled launches ran
(from the bench's own JSON line in the kernel-trace pass) is recorded, so the bench
cites the profile only for the schedule it times.

Only launches of the timed kernel with the timed grid count: the mean kernel
duration is taken over those dispatches in the kernel trace."""
import collections
import csv
import glob
import json
import os
import shutil
import sys

src, tag = sys.argv[1], sys.argv[2]
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = sys.argv[3] if len(sys.argv) > 3 else os.path.join(repo, "profiles")   # the GPU box: under gpurun_out/
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))


def grid_of(row):
    """Grid size in threads of a kernel-trace or counter-collection row (the two CSVs name it differently)."""
    return int(row["Grid_Size"]) if "Grid_Size" in row else int(row["Grid_Size_X"])


def bench_line(log):
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    return None


line = bench_line(os.path.join(src, "bench_kt.log"))
sched = None
if os.path.exists(os.path.join(src, "bench_kt_detail.json")):   # round 4+: the schedule is in the detail file
    with open(os.path.join(src, "bench_kt_detail.json")) as f:
        sched = json.load(f)["head"]["schedule"]
elif line and "detail" in line:
    sched = line["detail"]["schedule"]
grid = sched["grid_waves"] * 64 if sched else None

# the timed kernel = the trace_kernel instantiation with the most calls; its dispatches at the timed grid
stats = list(csv.DictReader(open(os.path.join(src, "kt", "run_kernel_stats.csv"))))
timed = max((r for r in stats if "trace_kernel" in r["Name"]), key=lambda r: int(r["Calls"]))
durs = []
for f in glob.glob(os.path.join(src, "kt", "run_kernel_trace.csv")):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"] == timed["Name"] and (grid is None or grid_of(r) == grid):
            durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = {"kernel": timed["Name"], "calls": int(timed["Calls"]), "avg_ns_all_calls": float(timed["AverageNs"]),
       "timed_grid_calls": len(durs), "avg_ns": (sum(durs) / len(durs)) if durs else float(timed["AverageNs"]),
       "min_ns": float(timed["MinNs"]), "max_ns": float(timed["MaxNs"]), "schedule": sched,
       "bench_value": line["value"] if line else None, "pmc": {}}
for p in sorted(d for d in os.listdir(src) if d.startswith("pmc")):
    rows = list(csv.DictReader(open(os.path.join(src, p, "run_counter_collection.csv"))))
    vals = collections.defaultdict(list)
    for r in rows:
        if r["Kernel_Name"] == timed["Name"] and (grid is None or grid_of(r) == grid):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            out.update({"grid_size": grid_of(r), "lds": int(r["LDS_Block_Size"])})
    for k, v in vals.items():
        out["pmc"][k] = {"per_launch_mean": sum(v) / len(v), "launches": len(v)}
pm = {k: v["per_launch_mean"] for k, v in out["pmc"].items()}
need = ("TCP_TCC_READ_REQ_sum", "TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "WRITE_SIZE")
if all(k in pm for k in need):
    rd = (pm["TCC_EA0_RDREQ_sum"] - pm["TCC_EA0_RDREQ_32B_sum"]) * 128 + pm["TCC_EA0_RDREQ_32B_sum"] * 32
    out["levels"] = {"l2_request_bytes": pm["TCP_TCC_READ_REQ_sum"] * 128, "fabric_read_bytes": rd,
                     "write_bytes": pm["WRITE_SIZE"] * 1024, "fabric_bytes": rd + pm["WRITE_SIZE"] * 1024}
if all(k in pm for k in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "GRBM_GUI_ACTIVE")):
    # busy cycles per CU per kernel cycle (GRBM_GUI_ACTIVE counts every XCD's clock: / 8 XCDs;
    # one TA and one TD per CU, 256 CUs): the vector-memory path's utilisation (bench vmem_frac)
    cyc = pm["GRBM_GUI_ACTIVE"] / 8
    out["vmem"] = {"ta_busy_frac": pm["TA_TA_BUSY_sum"] / 256 / cyc, "td_busy_frac": pm["TD_TD_BUSY_sum"] / 256 / cyc,
                   "kernel_cycles": cyc}
if "TCC_HIT_sum" in pm and "TCC_MISS_sum" in pm:
    out["l2_hit_rate"] = pm["TCC_HIT_sum"] / (pm["TCC_HIT_sum"] + pm["TCC_MISS_sum"])
json.dump(out, open(os.path.join(dst, f"{tag}_pmc_summary.json"), "w"), indent=1)
print(json.dumps({k: out.get(k) for k in ("kernel", "avg_ns", "timed_grid_calls", "schedule", "levels", "l2_hit_rate",
                                          "vmem")}))
