#!/bin/bash
# Counter calibration for the per-level roofline (tools/ubench_levels.hip): the
# list of available counters, one plain run (times), then one rocprofv3 --pmc
# pass per counter group, each under its own time limit. Output: gpurun_out/calib/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/calib
mkdir -p $OUT
timeout -k 10 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || echo "list-avail failed"
timeout -k 10 60 tools/ubench_levels > $OUT/plain.txt 2>&1 || { echo "plain run failed"; cat $OUT/plain.txt; exit 1; }
cat $OUT/plain.txt
i=0
for set in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_READ_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
           "FETCH_SIZE" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
           "TCC_EA0_RDREQ_DRAM_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" \
           "TA_BUFFER_READ_WAVEFRONTS_sum TA_BUSY_avr GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- tools/ubench_levels > $OUT/log$i 2>&1 \
    && echo "pass $i ok: $set" || echo "pass $i failed: $set"
done
python3 - <<'PY'
import csv, glob, collections
rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob("gpurun_out/calib/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        rows[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(rows):
    if "levels_kernel" not in k:
        continue
    print(k)
    for c in sorted(rows[k]):
        v = rows[k][c]
        print(f"   {c:36s} {sum(v)/len(v):18.1f}")
PY
