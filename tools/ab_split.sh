#!/bin/bash
# A/B: in-wave stack splitting (MRT_SPLIT_LIVE: live-lane count of a wave's last round that triggers it).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V="--variant lib/variants/split0:{} --variant lib:{}"
for v in split8 split32; do V="$V --variant lib/variants/$v:{}"; done
AB_WORKLOADS=${AB_WORKLOADS:-'bunny-primary-1024x768 bunny-primary-640x480 sponza-diffuse-640x480 conference-ao-640x480 hairball-diffuse-640x480 mori-primary-640x480'} \
  bash tools/ab_round.sh $V
