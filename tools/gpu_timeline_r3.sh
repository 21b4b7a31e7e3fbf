#!/bin/bash
# Frame timelines (tools/timeline.py, MRT_STATS_TIMELINE build) of the workloads whose tails bound the frame.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for W in ${TL_WORKLOADS:-hairball-diffuse-1920x1080 hairball-diffuse-640x480 bunny-primary-640x480}; do
MRT_LIB_DIR=$PWD/gpu-ray-tracing_amd/lib/variants/timeline timeout -k 10 300 python -u tools/timeline.py $W '{"autotune": 0}' > gpurun_out/tl_$W.txt 2> gpurun_out/tl_$W.err || { echo "failed $W"; tail gpurun_out/tl_$W.err; exit 1; }
cat gpurun_out/tl_$W.txt
done
