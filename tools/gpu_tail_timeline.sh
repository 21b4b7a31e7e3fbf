#!/bin/bash
# Tail diagnostics: correctness of the tail variants, the tail timeline (tools/tail_timeline.py with the
# MRT_TAIL_TIMELINE build) and the A/B of tail_lanes on the bench workloads (tools/ab_tail.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
rm -f gpurun_out/tail_tl.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "tail or comb or launch_configs or speculative" > gpurun_out/pytest_tail.log 2>&1 || { echo "pytest tail failed"; tail -40 gpurun_out/pytest_tail.log; exit 1; }
tail -1 gpurun_out/pytest_tail.log
for W in bunny-primary-640x480 hairball-diffuse-640x480; do
MRT_LIB_DIR=$PWD/gpu-ray-tracing_amd/lib/variants/tailtl timeout -k 10 300 python -u tools/tail_timeline.py $W '{"tail_lanes": 0, "autotune": 0}' '{"tail_lanes": 16, "autotune": 0}' >> gpurun_out/tail_tl.txt 2>> gpurun_out/tail_tl.err || { echo "failed $W"; tail gpurun_out/tail_tl.err; exit 1; }
done
cut -c1-300 gpurun_out/tail_tl.txt
timeout -k 10 900 python -u tools/ab_tail.py ${AB_ARGS} > gpurun_out/ab_tail.txt 2> gpurun_out/ab_tail.err || { echo "ab failed"; tail -20 gpurun_out/ab_tail.err; exit 1; }
cat gpurun_out/ab_tail.txt
