#!/bin/bash
# Round-3 parity + quick A/B of the cooperative tail (tail_lanes 0 vs 16) on the bench workloads.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "timed or overflow" > gpurun_out/pytest_tail.log 2>&1 || { echo "pytest tail failed"; tail -40 gpurun_out/pytest_tail.log; }
tail -2 gpurun_out/pytest_tail.log
timeout -k 10 900 python -u tools/ab_tail.py > gpurun_out/ab_tail.txt 2> gpurun_out/ab_tail.err || { echo "ab failed"; tail -20 gpurun_out/ab_tail.err; }
cat gpurun_out/ab_tail.txt
