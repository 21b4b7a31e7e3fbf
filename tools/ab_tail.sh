#!/bin/bash
# A/B: tail export thresholds — round age (lib) vs launch age (variants/kclock) — and the resume grid.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V="--variant lib:{\"tail_lanes\":-1}"
for c in '64,30,1,4' '64,30,2,4' '64,30,1,8' '16,40,1,4'; do
  IFS=, read k t l w <<< "$c"
  V="$V --variant lib:{\"tail_lanes\":$k,\"tail_after_us\":$t,\"tail_resume_lanes\":$l,\"tail_resume_waves\":$w}"
done
for c in '64,60,1,4' '64,60,4,4' '64,50,2,4' '32,50,1,8'; do
  IFS=, read k t l w <<< "$c"
  V="$V --variant lib/variants/kclock:{\"tail_lanes\":$k,\"tail_after_us\":$t,\"tail_resume_lanes\":$l,\"tail_resume_waves\":$w}"
done
AB_WORKLOADS=${AB_WORKLOADS:-'bunny-primary-1024x768 bunny-primary-640x480 sponza-diffuse-640x480 conference-ao-640x480 hairball-diffuse-640x480'} \
  bash tools/ab_round.sh $V
