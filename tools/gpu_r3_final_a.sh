#!/bin/bash
# Round 3: hairball knob sweep, steady-state schedule tuning over every schedule x modifier
# (tools/tune_db.py -> gpurun_out/tuned_schedules.json), then the bench locking those schedules.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_r3_sweep.sh || exit 1
timeout -k 10 900 python -u tools/tune_db.py --out gpurun_out/tuned_schedules.json > gpurun_out/tune_db.txt 2> gpurun_out/tune_db.err || { echo "tune_db failed"; tail -20 gpurun_out/tune_db.err; exit 1; }
cut -c1-500 gpurun_out/tune_db.txt
timeout -k 10 400 python bench.py --tune-db gpurun_out/tuned_schedules.json > gpurun_out/bench_t2.json 2> gpurun_out/bench_t2.err || { echo "bench failed"; tail -30 gpurun_out/bench_t2.err; exit 1; }
grep -E "extra|head|strong" gpurun_out/bench_t2.err
