#!/bin/bash
# Vector-memory pipeline counters for one bench workload: how busy the texture
# address (TA) / texture data (TD) units are against GRBM_GUI_ACTIVE, and how many
# buffer-load wave instructions reach them. Each pass is its own rocprofv3 run
# (counter limits per block: 2 TA, 2 TD, 2 GRBM, 4 TCP).
#   pmc_pipe.sh [workload] [outdir] [counter sets...]   (sets: space-separated names, ';' between passes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
W=${1:-hairball-diffuse-1920x1080}
OUT=${2:-gpurun_out/pipe}
SETS=${3:-"GRBM_GUI_ACTIVE TA_BUSY_avr TA_BUFFER_READ_WAVEFRONTS_sum;TD_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum GRBM_COUNT"}
B="--workload $W --no-extra --no-cpu --no-strong --bvh-cache /tmp/mrt_bvhcache"
mkdir -p $OUT
timeout -k 10 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || { echo "list-avail failed"; exit 1; }
timeout -k 10 300 python3 bench.py $B --steps 2 --warmup 1 > $OUT/bench_warm.log 2>&1 || { echo "warm run failed"; tail $OUT/bench_warm.log; exit 1; }
i=0
IFS=';' read -ra PASSES <<< "$SETS"
for P in "${PASSES[@]}"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 bench.py $B --steps 5 > $OUT/bench_p$i.log 2>&1 || { echo "pass $i ($P) failed"; tail -5 $OUT/bench_p$i.log; exit 1; }
    echo "pass $i ok: $P"
done
