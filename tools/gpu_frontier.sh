#!/bin/bash
# Frontier tail: its GPU parity tests, the A/B of tail_lanes 0/16 on the bench workloads and the tail timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "tail or comb or frontier or launch_configs" > gpurun_out/pytest_tail.log 2>&1 || { echo "pytest tail failed"; grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_tail.log | head -20; tail -30 gpurun_out/pytest_tail.log; exit 1; }
tail -1 gpurun_out/pytest_tail.log
timeout -k 10 600 python -u tools/ab_tail.py ${AB_ARGS} > gpurun_out/ab_tail.txt 2> gpurun_out/ab_tail.err || { echo "ab failed"; tail -20 gpurun_out/ab_tail.err; exit 1; }
cat gpurun_out/ab_tail.txt
for W in bunny-primary-640x480 hairball-diffuse-640x480; do
MRT_LIB_DIR=$PWD/gpu-ray-tracing_amd/lib/variants/tailtl timeout -k 10 300 python -u tools/tail_timeline.py $W '{"tail_lanes": 0, "autotune": 0}' '{"tail_lanes": 16, "autotune": 0}' >> gpurun_out/tail_tl.txt 2>> gpurun_out/tail_tl.err || { echo "failed $W"; tail gpurun_out/tail_tl.err; exit 1; }
done
cut -c1-400 gpurun_out/tail_tl.txt
