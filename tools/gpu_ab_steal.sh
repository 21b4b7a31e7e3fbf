#!/bin/bash
# A/B of the queue schedules with and without stealing (tools/ab_tail.py), hairball and bunny batches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
G='"num_queues": 1, "fetch_threshold": 48, "autotune": 0'
Q='"num_queues": 8, "fetch_threshold": 48, "autotune": 0'
timeout -k 10 900 python -u tools/ab_tail.py --rounds 5 --workload hairball-diffuse-1920x1080 --workload hairball-diffuse-640x480 \
  --config "{$G, \"waves_per_cu\": 16}" --config "{$Q, \"waves_per_cu\": 16, \"steal\": 1}" \
  --config "{$Q, \"waves_per_cu\": 16, \"steal\": 0}" --config "{$Q, \"waves_per_cu\": 12, \"steal\": 1}" \
  --config "{$Q, \"waves_per_cu\": 20, \"steal\": 1}" > gpurun_out/ab_steal.txt 2> gpurun_out/ab_steal.err || { echo "ab failed"; tail -20 gpurun_out/ab_steal.err; exit 1; }
timeout -k 10 600 python -u tools/ab_tail.py --rounds 5 --workload bunny-primary-1024x768 --workload bunny-primary-640x480 --workload sponza-diffuse-640x480 \
  --config '{"autotune": 0}' --config '{"num_queues": 8, "waves_per_cu": 8, "autotune": 0}' \
  --config '{"num_queues": 8, "waves_per_cu": 8, "autotune": 0, "steal": 1}' \
  --config '{"num_queues": 8, "waves_per_cu": 20, "autotune": 0, "steal": 1}' >> gpurun_out/ab_steal.txt 2>> gpurun_out/ab_steal.err || { echo "ab2 failed"; tail -20 gpurun_out/ab_steal.err; exit 1; }
cat gpurun_out/ab_steal.txt
