#!/bin/bash
# A/B rounds of tools/ab.py over the bench workloads; output in gpurun_out/ab.log.
cd "$GRAFT_REPO_ROOT" || exit 1
: > gpurun_out/ab.log
for W in ${AB_WORKLOADS:-bunny-primary-1024x768 bunny-primary-640x480 sponza-diffuse-640x480 conference-ao-640x480}; do
  timeout -k 10 300 python -u tools/ab.py --workload $W "$@" >> gpurun_out/ab.log 2>&1 || { echo "ab failed on $W"; tail -20 gpurun_out/ab.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/ab.log
