#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
V="--variant lib/variants/r2:{\"autotune\":0} --variant lib/variants/notail:{\"autotune\":0}
   --variant lib:{\"autotune\":0,\"tail_lanes\":0} --variant lib:{\"autotune\":0,\"tail_lanes\":16}"
timeout -k 10 900 python -u tools/ab.py --rounds 7 --launches 30 --workload conference-ao-640x480 --workload bunny-primary-1024x768 \
   --workload bunny-primary-640x480 --workload sponza-diffuse-640x480 $V > gpurun_out/ab_r2b.txt 2> gpurun_out/ab_r2b.err || { echo "ab failed"; tail -20 gpurun_out/ab_r2b.err; exit 1; }
cat gpurun_out/ab_r2b.txt
