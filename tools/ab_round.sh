#!/bin/bash
# Interleaved A/B of variant libraries on the standard workloads (tools/ab.py). Usage: ab_round.sh VARIANT_SPEC...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
W=""
for w in ${AB_WORKLOADS:-bunny-primary-1024x768 bunny-primary-640x480 conference-ao-640x480 sponza-diffuse-640x480 hairball-diffuse-640x480 hairball-diffuse-1920x1080}; do W="$W --workload $w"; done
V=""
for v in "$@"; do V="$V --variant $v"; done
timeout -k 10 900 python tools/ab.py $W $V 2>&1 | grep -v amdgpu.ids
