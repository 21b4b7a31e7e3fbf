#!/bin/bash
# Memory-pipeline counters (TA / TD / TCP / TCC) for one workload, one
# --pmc pass per group, no trace domains. Usage: pmc_mem.sh [workload] [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/pmcm
mkdir -p $OUT
W=${1:-bunny-primary-1024x768}
shift
rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
i=0
for set in "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE" \
           "TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
           "TCP_TA_TCP_STATE_READ_sum TCP_TOTAL_READ_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
           "TA_BUSY_max TA_BUSY_min TA_BUSY_avr"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 bench.py --workload $W --no-extra --no-cpu --steps 5 "$@" > $OUT/log$i 2>&1 || { echo "pass $i ($set) failed"; grep -i "error\|invalid\|not found" $OUT/log$i | head -3; }
done
python3 - <<'PY'
import csv, glob, collections
rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmcm/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "trace_kernel<" in r["Kernel_Name"]:
            rows[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
name = max(rows, key=lambda k: max(len(v) for v in rows[k].values()))   # the timed kernel: most dispatches
print(name)
for k in sorted(rows[name]):
    v = rows[name][k]
    print(f"{k:40s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
