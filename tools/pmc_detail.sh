#!/bin/bash
# Stall / instruction-mix counters for the headline workload (separate --pmc passes, no trace domains).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/pmcd
mkdir -p $OUT
W=${1:-bunny-primary-1024x768}
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SMEM" "SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 bench.py --workload $W --no-extra --no-cpu --steps 5 > $OUT/log$i 2>&1 || { echo "pass $i failed"; tail -5 $OUT/log$i; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmcd/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "trace_kernel<16, false, true, true, false, false, false>" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    v = agg[k]
    print(f"{k:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
