#!/bin/bash
# A/B: shallow-stack pop reads issued with the node loads (MRT_EARLY_LDS).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
AB_WORKLOADS=${AB_WORKLOADS:-'bunny-primary-1024x768 bunny-primary-640x480 sponza-diffuse-640x480 conference-ao-640x480 hairball-diffuse-640x480 bunny-primary-1920x1080'} \
  bash tools/ab_round.sh --variant lib:{} --variant lib/variants/early:{} --rounds 7
