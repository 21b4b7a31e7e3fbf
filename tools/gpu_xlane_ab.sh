#!/bin/bash
# A/B of the frontier tail's cross-lane ops: permlane swaps / readlane (MRT_TAIL_XLANE=1) vs LDS permutes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab.py --rounds 7 --launches 30 --workload hairball-diffuse-1920x1080 --workload hairball-diffuse-640x480 \
  --workload mori-ao-640x480 --workload bunny-primary-640x480 --workload conference-ao-640x480 \
  --variant 'lib:{"saved":1}' --variant 'lib/variants/xl0:{"saved":1}' --variant 'lib:{"autotune":0}' --variant 'lib/variants/xl0:{"autotune":0}' \
  > gpurun_out/ab_xlane.txt 2> gpurun_out/ab_xlane.err || { echo "ab failed"; tail -20 gpurun_out/ab_xlane.err; exit 1; }
cat gpurun_out/ab_xlane.txt
