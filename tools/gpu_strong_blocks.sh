#!/bin/bash
# Strong-scaling shard block size: per-shard times projected on one GPU for several block-cyclic block sizes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for B in ${BLOCKS:-16384 4096 1024 256}; do
  timeout -k 10 300 python bench.py --no-extra --no-cpu --no-fast --no-explore --steps 20 --strong-steps 20 --strong-block $B --detail-out gpurun_out/strong_b$B.json > gpurun_out/strong_b$B.out 2> gpurun_out/strong_b$B.err || { echo "block $B failed"; tail -5 gpurun_out/strong_b$B.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/strong_b$B.json'))['strong']
print('block $B T1', d['t1_ms'], {k: (v['eta'], [round(x,3) for x in v['shard_ms']]) for k, v in d['projected_from_one_gpu'].items()})"
done
