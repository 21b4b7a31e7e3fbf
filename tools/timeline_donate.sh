cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export MRT_LIB_DIR=$PWD/gpu-ray-tracing_amd/lib/variants/timeline
TL_TAG=_off timeout -k 10 200 python tools/timeline.py bunny-primary-1024x768 '{"donate_lanes":-1}' > gpurun_out/timeline_off.log 2>&1 &&
TL_TAG=_d16 timeout -k 10 200 python tools/timeline.py bunny-primary-1024x768 '{"donate_lanes":16}' > gpurun_out/timeline_d16.log 2>&1
