#!/bin/bash
# Runs bench.py (no CPU leg, no extras, no strong scaling) once per argument set and prints one summary line each.
# Usage: sweep_bench.sh "--workload X --lane-groups 1" "--workload X --lane-groups 8" ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sweep
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 240 python bench.py --no-cpu --no-extra --no-strong --steps 50 $args > gpurun_out/sweep/b$i.json 2> gpurun_out/sweep/b$i.err || { echo "FAILED: $args"; tail -3 gpurun_out/sweep/b$i.err; exit 1; }
  python - "$args" gpurun_out/sweep/b$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:60s} {d['value']:9.1f} Mrays/s  kernel {d['detail']['kernel_ms_per_launch']:.4f} ms  step {d['ms_per_step']:.4f} ms", flush=True)
PY
done
