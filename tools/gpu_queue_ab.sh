#!/bin/bash
# Round 4 queue A/B: parity subset, then round 3 vs the tree (with and without the per-XCD queue shares
# code) on the rule schedules and the per-XCD queue forms, then PMC passes of the hairball 2 M-ray batch.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "wide_lists or two_handles or frontier_tail or known_answers or launch_configs" > gpurun_out/pytest_q.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/pytest_q.log | head -20; tail -30 gpurun_out/pytest_q.log; exit 1; }
tail -1 gpurun_out/pytest_q.log
Q='"num_queues":8,"fetch_threshold":48'
CFGS=('{"autotune":0}'
      "{\"autotune\":0,$Q,\"queue_shared\":10,\"queue_block\":16384,\"waves_per_cu\":16}"
      "{\"autotune\":0,$Q,\"queue_shared\":10,\"queue_block\":16384,\"waves_per_cu\":20}"
      "{\"autotune\":0,$Q,\"queue_shared\":5,\"queue_block\":4096,\"waves_per_cu\":20}"
      "{\"autotune\":0,$Q,\"queue_shared\":10,\"queue_block\":65536,\"waves_per_cu\":16}"
      '{"autotune":0,"num_queues":1,"fetch_threshold":48,"waves_per_cu":20,"lane_groups":16}')
V=""
for c in "${CFGS[@]}"; do V="$V --variant lib:$c"; done
timeout -k 10 900 python -u tools/ab.py --rounds 5 --launches 20 --workload hairball-diffuse-1920x1080 --workload hairball-diffuse-640x480 \
  --workload bunny-primary-1024x768 --workload bunny-primary-640x480 --workload mori-ao-640x480 --workload conference-ao-640x480 \
  --workload sponza-diffuse-640x480 --variant 'lib/variants/r3:{"autotune":0}' --variant 'lib/variants/noshares:{"autotune":0}' $V \
  > gpurun_out/ab_q.txt 2> gpurun_out/ab_q.err || { echo "ab failed"; tail -20 gpurun_out/ab_q.err; exit 1; }
cat gpurun_out/ab_q.txt
timeout -k 10 900 bash tools/pmc_configs.sh hairball-diffuse-1920x1080 "${CFGS[@]}" > gpurun_out/pmc_cfg.txt 2>&1 || { echo "pmc failed"; tail gpurun_out/pmc_cfg.txt; exit 1; }
cat gpurun_out/pmc_cfg.txt
