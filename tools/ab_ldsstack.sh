#!/bin/bash
# A/B: traversal-stack entries kept in LDS per lane (8 / 16 / 32; the rest spills to HBM).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
AB_WORKLOADS=${AB_WORKLOADS:-'bunny-primary-1024x768 bunny-primary-640x480 sponza-diffuse-640x480 conference-ao-640x480 hairball-diffuse-640x480 bunny-primary-1920x1080'} \
  bash tools/ab_round.sh --variant lib:{} --variant 'lib:{"lds_stack":8}' --variant 'lib:{"lds_stack":32}'
