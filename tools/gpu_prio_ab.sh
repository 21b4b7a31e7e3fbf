#!/bin/bash
# A/B of wave priority in the drain: MRT_TAIL_PRIO (frontier tail) and MRT_DRAIN_PRIO (waves that can no longer refill).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
X='"autotune":0,"num_queues":8,"fetch_threshold":48,"waves_per_cu":20,"queue_shared":5,"queue_block":16384'
timeout -k 10 500 python -u tools/ab.py --workload hairball-diffuse-1920x1080 --workload conference-ao-640x480 --workload mori-ao-640x480 --workload bunny-primary-1024x768 --workload sponza-diffuse-640x480 \
  --variant "lib/variants/base:{$X}" --variant "lib/variants/tprio:{$X}" --variant "lib/variants/dprio:{$X}" \
  --variant 'lib/variants/base:{"autotune":0}' --variant 'lib/variants/tprio:{"autotune":0}' --variant 'lib/variants/dprio:{"autotune":0}' > gpurun_out/prio_ab.txt 2> gpurun_out/prio_ab.err
