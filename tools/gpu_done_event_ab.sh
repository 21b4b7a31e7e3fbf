#!/bin/bash
# Cost of a completion event after every launch (-DMRT_DONE_EVENT: handle-scoped waits) on back-to-back launches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab.py --rounds 7 --launches 30 --workload conference-ao-640x480 --workload mori-ao-640x480 \
  --workload bunny-primary-640x480 --workload bunny-primary-1024x768 --workload hairball-diffuse-1920x1080 \
  --variant 'lib:{"saved":1}' --variant 'lib/variants/doneev:{"saved":1}' --variant 'lib:{"autotune":0}' --variant 'lib/variants/doneev:{"autotune":0}' > gpurun_out/ab_done.txt 2> gpurun_out/ab_done.err || { echo "ab failed"; tail -20 gpurun_out/ab_done.err; exit 1; }
cat gpurun_out/ab_done.txt
