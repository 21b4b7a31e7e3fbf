#!/bin/bash
# Profiles every bench workload (tools/profile_round.sh each); outputs under gpurun_out/prof_<workload>.
cd "$GRAFT_REPO_ROOT" || exit 1
for W in "$@"; do
  bash tools/profile_round.sh $W gpurun_out/prof_$W > gpurun_out/prof_$W.log 2>&1 || { echo "profile $W failed"; tail -5 gpurun_out/prof_$W.log; exit 1; }
  echo "profiled $W"
done
