#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for ML in 1 2 3 4; do
  timeout -k 10 300 python bench.py --no-extra --no-cpu --no-fast --no-explore --steps 20 --strong-min-launches $ML --detail-out gpurun_out/strong_ml$ML.json > gpurun_out/strong_ml$ML.out 2> gpurun_out/strong_ml$ML.err || { echo "ml $ML failed"; tail -5 gpurun_out/strong_ml$ML.err; exit 1; }
  echo "min_launches $ML: $(grep strong gpurun_out/strong_ml$ML.err)"
done
