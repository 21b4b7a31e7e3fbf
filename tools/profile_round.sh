#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats of one bench workload,
# then separate PMC passes (FETCH_SIZE, WRITE_SIZE, TCC hit/miss) — never
# combined with any trace domain. Usage: profile_round.sh [workload] [outdir]
# (summarize with tools/summarize_prof.py <outdir> <tag>).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
W=${1:-bunny-primary-1024x768}
OUT=${2:-gpurun_out/prof}
B="--workload $W --no-extra --no-cpu --no-strong --bvh-cache /tmp/mrt_bvhcache"
mkdir -p $OUT
# build (or load) the BVH once outside the profiler
timeout -k 10 300 python3 bench.py $B --steps 2 --warmup 1 > $OUT/bench_warm.log 2>&1 || { echo "warm run failed"; tail $OUT/bench_warm.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py $B --steps 20 > $OUT/bench_kt.log 2>&1 || { echo "kt failed"; tail $OUT/bench_kt.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc1 -o run -- python3 bench.py $B --steps 5 > $OUT/bench_pmc1.log 2>&1 || { echo "pmc1 failed"; tail $OUT/bench_pmc1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc2 -o run -- python3 bench.py $B --steps 5 > $OUT/bench_pmc2.log 2>&1 || { echo "pmc2 failed"; tail $OUT/bench_pmc2.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc3 -o run -- python3 bench.py $B --steps 5 > $OUT/bench_pmc3.log 2>&1 || { echo "pmc3 failed"; tail $OUT/bench_pmc3.log; exit 1; }
find $OUT -name "*.csv" | head -20
