#!/bin/bash
# Round 3 final (3/4): the bench line (saved schedules, citing the round-3 profiles).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { echo "bench failed"; tail -30 gpurun_out/bench_final.err; exit 1; }
grep -E "extra|head|strong" gpurun_out/bench_final.err
