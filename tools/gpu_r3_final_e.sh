#!/bin/bash
# Round 3 final (4/4): every README cell tuned and measured (tools/gpu_readme.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_readme.sh
