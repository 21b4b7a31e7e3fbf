#!/bin/bash
# Round 3 final (2/3): rocprofv3 kernel stats + PMC summaries of every bench workload under the saved schedules.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
# the 2 M-ray hairball batch (the 8-rank strong-scaling shard's size) with a 1.5 % margin: the global queue at
# 20 waves/CU is 2.2 % faster there in every steady-state run (profiles/round3_sweep_hairball_frontier.txt)
cp gpu-ray-tracing_amd/mrt/tuned_schedules.json gpurun_out/tuned_schedules.json
timeout -k 10 300 python -u tools/tune_db.py --workload hairball-diffuse-1920x1080 --margin 0.015 --out gpurun_out/tuned_schedules.json > gpurun_out/tune_db_hb.txt 2> gpurun_out/tune_db_hb.err || { echo "tune failed"; tail gpurun_out/tune_db_hb.err; exit 1; }
cut -c1-400 gpurun_out/tune_db_hb.txt
# the fast-reciprocal variant of the headline batch too (the bench line's rcp_fast block cites its profile)
timeout -k 10 300 python -u tools/tune_db.py --workload bunny-primary-1024x768 --fast-rcp --out gpurun_out/tuned_schedules.json > gpurun_out/tune_db_fast.txt 2> gpurun_out/tune_db_fast.err || { echo "tune fast failed"; tail gpurun_out/tune_db_fast.err; exit 1; }
cut -c1-400 gpurun_out/tune_db_fast.txt
cp gpurun_out/tuned_schedules.json gpu-ray-tracing_amd/mrt/tuned_schedules.json
timeout -k 10 1000 bash tools/profile_all.sh round3 ${PROF_WL:-bunny-primary-1024x768 fast:bunny-primary-1024x768 bunny-primary-640x480 conference-ao-640x480 sponza-diffuse-640x480 sponza-diffuse2-640x480 hairball-diffuse-640x480 hairball-diffuse-1920x1080} || exit 1
ls gpurun_out/profiles
