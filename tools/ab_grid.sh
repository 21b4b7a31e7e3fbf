#!/bin/bash
# A/B: work distribution and grid size (strided rounds vs per-XCD queues) per workload.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V="--variant lib:{}"
for c in '{"waves_per_cu":8}' '{"waves_per_cu":12}' '{"waves_per_cu":16}' '{"num_queues":8}' '{"num_queues":8,"waves_per_cu":8}' '{"num_queues":8,"waves_per_cu":12}' '{"num_queues":8,"waves_per_cu":16}'; do
  V="$V --variant lib:$c"
done
AB_WORKLOADS=${AB_WORKLOADS:-'bunny-primary-1024x768 bunny-primary-640x480 sponza-diffuse-640x480 conference-ao-640x480 hairball-diffuse-640x480'} \
  bash tools/ab_round.sh $V
