#!/bin/bash
# Tail timelines of the weakest README cell (Mori AO) and the bunny primary frame with its saved schedule.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
rm -f gpurun_out/tail_tl3.txt
MRT_LIB_DIR=$PWD/gpu-ray-tracing_amd/lib/variants/tailtl timeout -k 10 300 python -u tools/tail_timeline.py mori-ao-640x480 '{"tail_lanes": 0, "autotune": 0}' '{"tail_lanes": 16, "autotune": 0}' '{"tail_lanes": 16, "autotune": 0, "waves_per_cu": 12}' >> gpurun_out/tail_tl3.txt 2>> gpurun_out/tail_tl3.err || { echo "failed"; tail gpurun_out/tail_tl3.err; exit 1; }
MRT_LIB_DIR=$PWD/gpu-ray-tracing_amd/lib/variants/tailtl timeout -k 10 300 python -u tools/tail_timeline.py bunny-primary-640x480 '{"tail_lanes": 16, "autotune": 0, "waves_per_cu": 16, "lane_groups": 16}' >> gpurun_out/tail_tl3.txt 2>> gpurun_out/tail_tl3.err || { echo "failed"; tail gpurun_out/tail_tl3.err; exit 1; }
cut -c1-500 gpurun_out/tail_tl3.txt
