#!/bin/bash
# Tail export/resume: single-launch check, A/B over workloads, then the GPU parity suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/tail_check.py bunny-primary-1024x768 '{"tail_lanes":-1}' '{"tail_lanes":16,"tail_after_us":30}' \
  '{"tail_lanes":64,"tail_after_us":1}' > gpurun_out/tail_check.log 2>&1 || { echo "tail_check failed"; cat gpurun_out/tail_check.log; exit 1; }
grep -v amdgpu.ids gpurun_out/tail_check.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "tail" --timeout 120 --timeout-method thread > gpurun_out/pytest_tail.log 2>&1 || { echo "tail tests failed"; tail -30 gpurun_out/pytest_tail.log; exit 1; }
tail -2 gpurun_out/pytest_tail.log
V="--variant lib:{\"tail_lanes\":-1}"
for kt in "8 20" "16 20" "16 40" "32 30" "64 30" "16 60"; do
  set -- $kt
  V="$V --variant lib:{\"tail_lanes\":$1,\"tail_after_us\":$2}"
done
AB_WORKLOADS=${AB_WORKLOADS:-'bunny-primary-1024x768 bunny-primary-640x480 sponza-diffuse-640x480 conference-ao-640x480 hairball-diffuse-640x480'} \
  bash tools/ab_round.sh $V || exit 1
