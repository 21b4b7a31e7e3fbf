#!/bin/bash
# The big-BVH queue rule at 16 vs 20 waves/CU: the hairball 2M-ray batch and the strong-scaling projection.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
B="--workload hairball-diffuse-1920x1080 --no-extra --no-cpu --no-fast --no-explore --steps 50"
for V in lib lib/variants/bq20 lib lib/variants/bq20; do
  MRT_LIB_DIR=$PWD/gpu-ray-tracing_amd/$V timeout -k 10 400 python bench.py $B > gpurun_out/bq.json 2> gpurun_out/bq.err || { echo "bench $V failed"; tail -20 gpurun_out/bq.err; exit 1; }
  echo "$V: $(grep -E 'head|strong' gpurun_out/bq.err | tr '\n' ' ')"
done
