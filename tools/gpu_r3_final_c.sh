#!/bin/bash
# Round 3 final (2/3): rocprofv3 kernel stats + PMC summaries of every bench workload under the saved
# schedules (gpu-ray-tracing_amd/mrt/tuned_schedules.json, which the bench locks).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1150 bash tools/profile_all.sh round3 ${PROF_WL:-bunny-primary-1024x768 fast:bunny-primary-1024x768 bunny-primary-640x480 conference-ao-640x480 sponza-diffuse-640x480 sponza-diffuse2-640x480 hairball-diffuse-640x480 hairball-diffuse-1920x1080} || exit 1
ls gpurun_out/profiles
