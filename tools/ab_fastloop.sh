#!/bin/bash
# A/B: shallow-stack node loop (MRT_FAST_LOOP) and scalar triangle math (-fno-slp-vectorize, fewer VGPRs).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V="--variant lib:{}"
V="$V --variant lib/variants/fastloop:{}"
V="$V --variant lib/variants/noslp:{}"
V="$V --variant lib/variants/fastloop_noslp:{}"
V="$V --variant lib/variants/fastloop_noslp:{\"waves_per_cu\":20}"
AB_WORKLOADS=${AB_WORKLOADS:-'bunny-primary-1024x768 bunny-primary-640x480 sponza-diffuse-640x480 conference-ao-640x480 hairball-diffuse-640x480'} \
  bash tools/ab_round.sh $V
