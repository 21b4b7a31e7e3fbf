#!/bin/bash
# L1->L2 lines, L2 hit rate and fabric lines per launch of one workload under several launch
# configs: one rocprofv3 --pmc pass per config (counters only, no trace domain) around
# tools/ab_tail.py's launches of that config. Usage: pmc_configs.sh WORKLOAD CONFIG_JSON...
# Output: gpurun_out/pmc_cfg/<i>/ and one summary line per config (tools/pmc_configs.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
W=$1; shift
OUT=gpurun_out/pmc_cfg_$W
mkdir -p $OUT
# build (or load) the BVH once outside the profiler
timeout -k 10 300 python3 tools/ab_tail.py --workload $W --config '{"autotune":0}' --rounds 1 --launches 2 > $OUT/warm.log 2>&1 || { echo "warm failed"; tail $OUT/warm.log; exit 1; }
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d $OUT/c$i -o run -- \
    python3 tools/ab_tail.py --workload $W --config "$C" --rounds 2 --launches 10 > $OUT/c$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/c$i.log; exit 1; }
  python3 tools/pmc_configs.py $OUT/c$i "$C" "$(grep -o '[0-9.]* ms' $OUT/c$i.log | head -1)" || exit 1
done
