#!/bin/bash
# Strong-scaling shards (8 ranks, one GPU) under per-XCD queue variants: the spread of the shard times.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B='"autotune":0,"num_queues":8,"fetch_threshold":48,"waves_per_cu":20'
export EXTRA_SCHEDS="sh5b4096={$B,\"queue_shared\":5,\"queue_block\":4096};sh15b4096={$B,\"queue_shared\":15,\"queue_block\":4096};sh30b4096={$B,\"queue_shared\":30,\"queue_block\":4096};sh5b1024={$B,\"queue_shared\":5,\"queue_block\":1024};sh15b1024={$B,\"queue_shared\":15,\"queue_block\":1024};sh5b16384={$B,\"queue_shared\":5,\"queue_block\":16384};sh10b256={$B,\"queue_shared\":10,\"queue_block\":256}"
export SCHEDS=sh5b4096,sh15b4096,sh30b4096,sh5b1024,sh15b1024,sh5b16384,sh10b256 ORDERS=fwd REPS=7
timeout -k 10 600 python -u tools/strong_diag.py > gpurun_out/shard_sweep.txt 2> gpurun_out/shard_sweep.err
