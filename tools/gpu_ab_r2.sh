#!/bin/bash
# The round-2 library against the current one (tools/ab.py, interleaved in one process), fixed schedules.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
V="--variant lib/variants/r2:{\"autotune\":0} --variant lib/variants/r2:{\"autotune\":0,\"spec_slack\":4}
   --variant lib:{\"autotune\":0,\"tail_lanes\":0} --variant lib:{\"autotune\":0,\"tail_lanes\":16}
   --variant lib:{\"autotune\":0,\"spec_slack\":4,\"tail_lanes\":0} --variant lib:{\"autotune\":0,\"spec_slack\":4,\"tail_lanes\":16}"
timeout -k 10 900 python -u tools/ab.py --rounds 7 --launches 30 --workload conference-ao-640x480 --workload bunny-primary-1024x768 \
   --workload bunny-primary-640x480 --workload sponza-diffuse-640x480 --workload mori-ao-640x480 $V > gpurun_out/ab_r2.txt 2> gpurun_out/ab_r2.err || { echo "ab failed"; tail -20 gpurun_out/ab_r2.err; exit 1; }
cat gpurun_out/ab_r2.txt
bash tools/gpu_ab_steal.sh
