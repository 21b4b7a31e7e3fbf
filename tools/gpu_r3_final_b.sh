#!/bin/bash
# Round 3 final (1/2): all GPU tests, steady-state tuning of the bench workloads (every schedule x
# modifier, tools/tune_db.py -> gpurun_out/tuned_schedules.json), the bench locking them.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log | head; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 900 python -u tools/tune_db.py --out gpurun_out/tuned_schedules.json > gpurun_out/tune_db.txt 2> gpurun_out/tune_db.err || { echo "tune_db failed"; tail -20 gpurun_out/tune_db.err; exit 1; }
cut -c1-500 gpurun_out/tune_db.txt
timeout -k 10 400 python bench.py --tune-db gpurun_out/tuned_schedules.json > gpurun_out/bench_t3.json 2> gpurun_out/bench_t3.err || { echo "bench failed"; tail -30 gpurun_out/bench_t3.err; exit 1; }
grep -E "extra|head|strong" gpurun_out/bench_t3.err
