#!/bin/bash
# A/B of the quantized 64-B wide nodes (cfg.wide = 2) against the exact 128-B ones on the TD-bound hairball
# frames, under the per-XCD schedule and the rule.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
X='"autotune":0,"num_queues":8,"fetch_threshold":48,"waves_per_cu":20,"spec_slack":6,"queue_shared":5,"queue_block":8192'
timeout -k 10 500 python -u tools/ab.py --rounds 7 --launches 30 --workload hairball-diffuse-1920x1080 --workload hairball-diffuse-640x480 \
  --workload hairball-primary-1024x768 \
  --variant "lib:{$X}" --variant "lib:{$X,\"wide\":2}" --variant 'lib:{"autotune":0}' --variant 'lib:{"autotune":0,"wide":2}' \
  > gpurun_out/ab_wideq.txt 2> gpurun_out/ab_wideq.err || { echo "ab failed"; tail -5 gpurun_out/ab_wideq.err; exit 1; }
cat gpurun_out/ab_wideq.txt
