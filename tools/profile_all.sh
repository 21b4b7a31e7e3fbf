#!/bin/bash
# Profiles bench workloads (tools/profile_round.sh each) and condenses each into
# gpurun_out/profiles/<tag>_<workload>[_rcpfast]_{kernel_stats.csv,pmc_summary.json}
# (copy them into profiles/). Usage: profile_all.sh TAG W1 W2 ... [fast:W ...]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
mkdir -p gpurun_out/profiles
for W in "$@"; do
  EXTRA=""; NAME=$W
  case $W in fast:*) W=${W#fast:}; EXTRA="--rcp fast"; NAME=${W}_rcpfast;; esac
  bash tools/profile_round.sh $W gpurun_out/prof_$NAME $EXTRA > gpurun_out/prof_$NAME.txt 2>&1 || { echo "profile $NAME failed"; tail -5 gpurun_out/prof_$NAME.txt; exit 1; }
  python3 tools/summarize_prof.py gpurun_out/prof_$NAME ${TAG}_$NAME gpurun_out/profiles | cut -c1-300 || { echo "summary $NAME failed"; exit 1; }
done
