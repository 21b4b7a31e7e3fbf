#!/bin/bash
# Lane groups (a wave's lanes take rays from 2^k distant image regions) with the frontier tail (tools/ab_tail.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
C=()
for L in 1 2 4 8 16; do C+=(--config "{\"autotune\":0,\"lane_groups\":$L}"); done
C+=(--config "{\"autotune\":0,\"lane_groups\":4,\"waves_per_cu\":12}")
timeout -k 10 800 python -u tools/ab_tail.py --workload bunny-primary-640x480 --workload bunny-primary-1024x768 --workload mori-ao-640x480 \
  --workload conference-ao-640x480 --workload sponza-diffuse-640x480 "${C[@]}" > gpurun_out/lanegroups.txt 2> gpurun_out/lanegroups.err || { echo "ab failed"; tail -20 gpurun_out/lanegroups.err; exit 1; }
sed 's/  |  /\n    /g' gpurun_out/lanegroups.txt
