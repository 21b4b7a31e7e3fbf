#!/bin/bash
# Render primary / AO / diffuse frames on the GPU box (tools/render_frame.py); every step bounded.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/frames
for spec in "bunny primary 1" "conference ao 8" "sponza diffuse 8" "mori ao 16"; do
  set -- $spec
  timeout -k 10 120 python tools/render_frame.py --scene $1 --ray-type $2 --samples $3 \
    --out gpurun_out/frames/$1-$2.ppm >> gpurun_out/frames/render.jsonl 2>> gpurun_out/frames/render.err || { tail -20 gpurun_out/frames/render.err; exit 1; }
done
cat gpurun_out/frames/render.jsonl
