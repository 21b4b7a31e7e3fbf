#!/bin/bash
# Launch-knob sweep of the production library (tools/ab.py, interleaved rounds).
#   ab_launch_sweep.sh "<workloads>" '<json cfg>' 'libdir:<json cfg>' ...
# (defaults: four BASELINE workloads; refill thresholds, queues, lane groups)
cd "$GRAFT_REPO_ROOT" || exit 1
W=${1:-bunny-primary-1024x768 sponza-diffuse-640x480 hairball-diffuse-640x480 conference-ao-640x480}
shift
CFGS=("$@")
if [ ${#CFGS[@]} -eq 0 ]; then
    CFGS=('{}' '{"fetch_threshold": 32}' '{"fetch_threshold": 48}' '{"fetch_threshold": 56}'
          '{"num_queues": 1, "fetch_threshold": 48}' '{"num_queues": 8, "fetch_threshold": 48}' '{"lane_groups": 4}')
fi
ARGS=()
for w in $W; do ARGS+=(--workload "$w"); done
for c in "${CFGS[@]}"; do case "$c" in "{"*) ARGS+=(--variant "lib:$c") ;; *) ARGS+=(--variant "$c") ;; esac; done
timeout -k 10 700 python tools/ab.py --warm-rounds ${WARM_ROUNDS:-1} "${ARGS[@]}" 2>&1 | grep -v amdgpu.ids
