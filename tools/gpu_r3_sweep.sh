#!/bin/bash
# Hairball refill threshold / waves per CU / tail threshold sweep with the frontier tail (tools/ab_tail.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
C=()
for T in 16 32 48 56; do C+=(--config "{\"autotune\":0,\"num_queues\":1,\"fetch_threshold\":$T,\"waves_per_cu\":16}"); done
for W in 12 20; do C+=(--config "{\"autotune\":0,\"num_queues\":1,\"fetch_threshold\":48,\"waves_per_cu\":$W}"); done
for L in 8 12; do C+=(--config "{\"autotune\":0,\"num_queues\":1,\"fetch_threshold\":48,\"waves_per_cu\":16,\"tail_lanes\":$L}"); done
timeout -k 10 800 python -u tools/ab_tail.py --workload hairball-diffuse-1920x1080 --workload hairball-diffuse-640x480 "${C[@]}" > gpurun_out/sweep_hb.txt 2> gpurun_out/sweep_hb.err || { echo "sweep failed"; tail -20 gpurun_out/sweep_hb.err; exit 1; }
sed 's/  |  /\n    /g' gpurun_out/sweep_hb.txt
