#!/bin/bash
# Workgroup size (MRT_BLOCK_THREADS 256 / 512 / 1024) on the short frames: the dispatch ramp of a one-round grid.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
V=""
for L in lib lib/variants/bt512 lib/variants/bt1024; do
  V="$V --variant $L:{\"autotune\":0} --variant $L:{\"autotune\":0,\"waves_per_cu\":16}"
done
timeout -k 10 800 python -u tools/ab.py --rounds 7 --launches 30 --workload mori-ao-640x480 --workload conference-ao-640x480 \
   --workload bunny-primary-640x480 --workload bunny-primary-1024x768 --workload sponza-diffuse-640x480 $V > gpurun_out/ab_bt.txt 2> gpurun_out/ab_bt.err || { echo "ab failed"; tail -20 gpurun_out/ab_bt.err; exit 1; }
cat gpurun_out/ab_bt.txt
