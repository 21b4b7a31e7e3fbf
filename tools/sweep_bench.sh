#!/bin/bash
# Runs bench.py (no CPU leg) once per argument set and prints one summary line each.
# Usage: sweep_bench.sh "--lane-groups 1" "--lane-groups 8" ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sweep
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 240 python bench.py --no-cpu $args > gpurun_out/sweep/b$i.json 2> gpurun_out/sweep/b$i.err || { echo "FAILED: $args"; tail -3 gpurun_out/sweep/b$i.err; exit 1; }
  python - "$args" gpurun_out/sweep/b$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ex = " ".join(f"{e['workload'].split('-')[0][:4]}{e['workload'].split('-')[1][:3]}={e['value']:.0f}" for e in d.get("extra_workloads", []))
print(f"{sys.argv[1]:40s} head={d['value']:.0f} ({d['detail']['kernel_ms_per_launch']:.4f} ms) {ex}", flush=True)
PY
done
