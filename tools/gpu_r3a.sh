#!/bin/bash
# Round-3 check: GPU tests, then a full bench run that autotunes every workload
# (no saved schedules) and writes the schedules it settled.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rA > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
grep -E "^(bunny|sponza|hairball|conference)" gpurun_out/pytest_gpu.log | head -20
timeout -k 10 600 python bench.py --tune-db '' --save-schedules gpurun_out/tuned_schedules.json > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err || { echo "bench failed"; tail -30 gpurun_out/bench_a.err; exit 1; }
grep -E "extra|head|strong|schedules" gpurun_out/bench_a.err
