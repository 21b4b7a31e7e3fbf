#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats of one bench workload, then
# one PMC pass per counter group (never combined with a trace domain):
#   TCP_TCC_READ_REQ  lines the L1s fetch from L2   (128 B each on gfx950)
#   TCC_HIT/TCC_MISS  L2 hit rate
#   TCC_EA0_RDREQ     lines L2 fetches over the fabric (Infinity Cache or HBM; 128 B, 32B-requests apart)
#   WRITE_SIZE        bytes written
#   TA_TA_BUSY/TD_TD_BUSY  the vector-memory path's address (TA) and data (TD) units busy, per CU
#                     cycle (round 6, VERDICT r5 #7: the unit the traversal actually saturates)
# The same command each time (the bench locks its saved schedules, so every pass runs
# the schedule the bench line times). Usage: profile_round.sh [workload] [outdir] [bench args...]
# (summarize with tools/summarize_prof.py <outdir> <tag>).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
W=${1:-bunny-primary-1024x768}
OUT=${2:-gpurun_out/prof}
shift 2
B="--workload $W --no-extra --no-cpu --no-strong --no-explore --no-fast --bvh-cache /tmp/mrt_bvhcache $*"
mkdir -p $OUT
# build (or load) the BVH once outside the profiler
timeout -k 10 300 python3 bench.py $B --steps 2 --warmup 1 > $OUT/bench_warm.log 2>&1 || { echo "warm run failed"; tail $OUT/bench_warm.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py $B --steps 50 --detail-out $OUT/bench_kt_detail.json > $OUT/bench_kt.log 2>&1 || { echo "kt failed"; tail $OUT/bench_kt.log; exit 1; }
i=0
for set in "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TCC_HIT_sum TCC_MISS_sum" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "WRITE_SIZE" "TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py $B --steps 10 > $OUT/bench_pmc$i.log 2>&1 || { echo "pmc$i ($set) failed"; tail -5 $OUT/bench_pmc$i.log; exit 1; }
done
echo "profiled $W"
