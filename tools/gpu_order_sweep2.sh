#!/bin/bash
# Strong-scaling shards, live blocks first: ordering granularity (dist blocks) x shared-queue share.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
B='"autotune":0,"num_queues":8,"fetch_threshold":48,"waves_per_cu":20,"spec_slack":6'
export EXTRA_SCHEDS="q8s5={$B,\"queue_block\":8192,\"queue_shared\":5};q8s10={$B,\"queue_block\":8192,\"queue_shared\":10};q8s20={$B,\"queue_block\":8192,\"queue_shared\":20};q16s10={$B,\"queue_block\":16384,\"queue_shared\":10}"
export SCHEDS=q8s5,q8s10,q8s20,q16s10 ORDERS=fwd REPS=7 ORDER=1
for BL in ${BLOCKS:-256 1024}; do
  BLOCK=$BL timeout -k 10 300 python -u tools/strong_diag.py > gpurun_out/order2_b${BL}.txt 2> gpurun_out/order2_b${BL}.err || { echo "diag $BL failed"; tail -5 gpurun_out/order2_b${BL}.err; exit 1; }
done
