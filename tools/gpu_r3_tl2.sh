#!/bin/bash
# Tail timeline of the hairball 2M-ray launch (the strong-scaling shard's size) and the A/B of tail thresholds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for W in hairball-diffuse-1920x1080 hairball-diffuse-640x480 bunny-primary-1024x768; do
MRT_LIB_DIR=$PWD/gpu-ray-tracing_amd/lib/variants/tailtl timeout -k 10 300 python -u tools/tail_timeline.py $W '{"tail_lanes": 0, "autotune": 0}' '{"tail_lanes": 16, "autotune": 0}' >> gpurun_out/tail_tl2.txt 2>> gpurun_out/tail_tl2.err || { echo "failed $W"; tail gpurun_out/tail_tl2.err; exit 1; }
done
cut -c1-400 gpurun_out/tail_tl2.txt
V="--variant lib/variants/r3a:{\"autotune\":0,\"tail_lanes\":16} --variant lib:{\"autotune\":0,\"tail_lanes\":16} --variant lib/variants/tspec:{\"autotune\":0,\"tail_lanes\":16}"
timeout -k 10 600 python -u tools/ab.py --rounds 7 --launches 30 --workload mori-ao-640x480 --workload bunny-primary-1024x768 \
   --workload bunny-primary-640x480 --workload hairball-diffuse-640x480 --workload hairball-diffuse-1920x1080 $V > gpurun_out/ab_loads.txt 2> gpurun_out/ab_loads.err || { echo "ab failed"; tail -20 gpurun_out/ab_loads.err; exit 1; }
cat gpurun_out/ab_loads.txt
