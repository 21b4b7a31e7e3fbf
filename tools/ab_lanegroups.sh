#!/bin/bash
# A/B: lane_groups (rays of a wave drawn from 2^k distant sub-ranges) per workload.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=""
for g in 1 4 16 64; do V="$V --variant lib:{\"lane_groups\":$g}"; done
AB_WORKLOADS=${AB_WORKLOADS:-'hairball-diffuse-640x480 sponza-diffuse-640x480 conference-diffuse-640x480 conference-ao-640x480 sponza-ao-640x480 bunny-primary-1024x768 bunny-primary-640x480'} \
  bash tools/ab_round.sh $V
