#!/bin/bash
# A/B: raise a wave's issue priority once its current round has run MRT_PRIO_AFTER_US (strided rounds).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
AB_WORKLOADS=${AB_WORKLOADS:-'bunny-primary-1024x768 bunny-primary-640x480 sponza-diffuse-640x480 conference-ao-640x480 hairball-diffuse-640x480 bunny-primary-1920x1080'} \
  bash tools/ab_round.sh --variant lib:{} --variant lib/variants/prio15:{} --variant lib/variants/prio40:{}
