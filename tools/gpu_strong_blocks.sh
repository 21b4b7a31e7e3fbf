#!/bin/bash
# Strong-scaling shard blocks: per-shard times projected on one GPU for several block sizes,
# blocks dealt cyclically (balance 0) or by live-ray count (balance 1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for BAL in ${BALANCE:-1 0}; do
for B in ${BLOCKS:-16384 4096 1024 256}; do
  T=b${B}_bal$BAL
  timeout -k 10 300 python bench.py --no-extra --no-cpu --no-fast --no-explore --steps 20 --strong-steps 20 --strong-block $B --strong-balance $BAL --detail-out gpurun_out/strong_$T.json > gpurun_out/strong_$T.out 2> gpurun_out/strong_$T.err || { echo "$T failed"; tail -5 gpurun_out/strong_$T.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/strong_$T.json'))['strong']
print('block $B balance $BAL T1', d['t1_ms'], 'one-stream', d.get('one_stream_ms'), {k: (v['eta'], [round(x,3) for x in v['shard_ms']]) for k, v in d['projected_from_one_gpu'].items()})"
done; done
