#!/bin/bash
# Round 3 final: the bench line (saved schedules, citing the round-3 profiles), then every README cell.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_r3_final_d.sh || exit 1
bash tools/gpu_readme.sh
