#!/bin/bash
# Round 3 close: every GPU test and the driver's smoke() on the committed tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_final.log 2>&1 || { echo "pytest failed"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu_final.log | head; tail -30 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || { echo "smoke failed"; exit 1; }
