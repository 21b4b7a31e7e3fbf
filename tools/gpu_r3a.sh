#!/bin/bash
# Round-3 check: GPU tests, the tail timeline, then a full bench run that autotunes every
# workload (no saved schedules) and writes the schedules it settled.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rA > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "^(FAILED|ERROR)|Error" gpurun_out/pytest_gpu.log | head; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
grep -E "^(bunny|sponza|hairball|conference)" gpurun_out/pytest_gpu.log | head -20
MRT_LIB_DIR=$PWD/gpu-ray-tracing_amd/lib/variants/tailtl timeout -k 10 300 python -u tools/tail_timeline.py bunny-primary-640x480 '{"tail_lanes": 16, "autotune": 0}' > gpurun_out/tail_tl.txt 2>> gpurun_out/tail_tl.err || { echo "timeline failed"; tail gpurun_out/tail_tl.err; exit 1; }
cut -c1-300 gpurun_out/tail_tl.txt
timeout -k 10 600 python bench.py --tune-db '' --save-schedules gpurun_out/tuned_schedules.json > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err || { echo "bench failed"; tail -30 gpurun_out/bench_a.err; exit 1; }
grep -E "extra|head|strong|schedules" gpurun_out/bench_a.err
