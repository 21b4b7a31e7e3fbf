#!/bin/bash
# A/B at 2 M-ray batches (1920x1080): occupancy (scalar triangle math: 77 VGPRs -> 24 waves/CU), distribution.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V="--variant lib:{}"
V="$V --variant lib/variants/noslp:{}"
V="$V --variant lib/variants/noslp:{\"waves_per_cu\":20}"
V="$V --variant lib:{\"num_queues\":8}"
V="$V --variant lib:{\"lane_groups\":4}"
AB_WORKLOADS=${AB_WORKLOADS:-'hairball-diffuse-1920x1080 bunny-primary-1920x1080 sponza-diffuse-1920x1080 conference-ao-1920x1080'} \
  bash tools/ab_round.sh $V
