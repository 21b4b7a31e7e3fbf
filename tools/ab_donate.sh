#!/bin/bash
# GPU tests, then A/B of sparse-wave if-if / lane donation settings against a saved build (lib/variants/base).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
V="--variant lib/variants/base:{}"
for c in '"ifif_lanes":-1' '"ifif_lanes":4' '"ifif_lanes":8' '"ifif_lanes":16' '"ifif_lanes":32' '"ifif_lanes":16,"donate_lanes":8'; do V="$V --variant lib:{$c}"; done
for c in '"ifif_lanes":-1' '"ifif_lanes":16'; do V="$V --variant lib/variants/w4:{$c}"; done
AB_WORKLOADS=${AB_WORKLOADS:-'bunny-primary-1024x768 bunny-primary-640x480 sponza-diffuse-640x480 conference-ao-640x480 hairball-diffuse-640x480'} \
  bash tools/ab_round.sh $V
