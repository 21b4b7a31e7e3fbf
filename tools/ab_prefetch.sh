#!/bin/bash
# A/B: prefetch touches (MRT_PREFETCH bit 0: pushed far child's node line; bit 1: postponed leaf's woop line).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V="--variant lib:{}"
for v in pf1 pf2 pf3; do V="$V --variant lib/variants/$v:{}"; done
AB_WORKLOADS=${AB_WORKLOADS:-'hairball-diffuse-640x480 sponza-diffuse-640x480 bunny-primary-1024x768 bunny-primary-640x480 conference-ao-640x480'} \
  bash tools/ab_round.sh $V
