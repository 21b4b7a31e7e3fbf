#!/bin/bash
# Two more bench runs of the committed tree (with profiles/round3_bench_n1.json: three runs on saved schedules).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 2 3; do
  timeout -k 10 400 python bench.py > gpurun_out/bench_det$i.json 2> gpurun_out/bench_det$i.err || { echo "bench $i failed"; tail -30 gpurun_out/bench_det$i.err; exit 1; }
  grep -E "head|strong" gpurun_out/bench_det$i.err
done
