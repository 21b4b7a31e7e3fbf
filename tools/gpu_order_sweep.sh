#!/bin/bash
# Strong-scaling shards with each shard's live blocks first (shard_spans priority): dist block size x
# balance x queue schedule, plus the 1 spp hairball frame under the candidate queue blocks.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
B='"autotune":0,"num_queues":8,"fetch_threshold":48,"waves_per_cu":20,"spec_slack":6,"queue_shared":5'
timeout -k 10 400 python -u tools/ab.py --rounds 7 --launches 30 --workload hairball-diffuse-1920x1080 \
  --variant "lib:{$B,\"queue_block\":4096}" --variant "lib:{$B,\"queue_block\":8192}" --variant "lib:{$B,\"queue_block\":16384}" \
  --variant "lib:{$B,\"queue_block\":16384,\"queue_shared\":10}" \
  > gpurun_out/ab_qblock.txt 2> gpurun_out/ab_qblock.err || { echo "ab failed"; tail -5 gpurun_out/ab_qblock.err; exit 1; }
cat gpurun_out/ab_qblock.txt
export EXTRA_SCHEDS="x4096={$B,\"queue_block\":4096};x8192={$B,\"queue_block\":8192};x16384={$B,\"queue_block\":16384}"
export SCHEDS=x4096,x8192,x16384 ORDERS=fwd REPS=7 ORDER=1
for BL in ${BLOCKS:-1024 4096}; do for BAL in 0 1; do
  BLOCK=$BL BALANCE=$BAL timeout -k 10 300 python -u tools/strong_diag.py > gpurun_out/order_b${BL}_bal$BAL.txt 2> gpurun_out/order_b${BL}_bal$BAL.err || { echo "diag $BL $BAL failed"; tail -5 gpurun_out/order_b${BL}_bal$BAL.err; exit 1; }
done; done
