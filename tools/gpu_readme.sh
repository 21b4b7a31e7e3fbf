#!/bin/bash
# Steady-state schedule tuning of every README cell (merged into a copy of the package's saved
# schedules), then the README table with them.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
cp gpu-ray-tracing_amd/mrt/tuned_schedules.json gpurun_out/tuned_schedules_all.json
W=$(python3 -c "import sys; sys.path.insert(0,'tools'); import readme_table as r; print(' '.join('--workload '+c[0] for c in r.CELLS))")
timeout -k 10 900 python -u tools/tune_db.py $W --rounds 2 --launches 10 --out gpurun_out/tuned_schedules_all.json > gpurun_out/tune_db_readme.txt 2> gpurun_out/tune_db_readme.err || { echo "tune failed"; tail -20 gpurun_out/tune_db_readme.err; exit 1; }
cut -c1-200 gpurun_out/tune_db_readme.txt
timeout -k 10 900 python -u tools/readme_table.py --tune-db gpurun_out/tuned_schedules_all.json > gpurun_out/readme_table.log 2>&1 || { echo "readme failed"; tail -20 gpurun_out/readme_table.log; exit 1; }
cat gpurun_out/readme_table.md
