#!/bin/bash
# One GPU-box session: parity tests, smoke, bench; every GPU step bounded.
# GPU_ROUND_GLOO=1 also rehearses the N=2 sharded flow (two ranks on the one GPU, gloo collectives).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
tail -c 600 gpurun_out/bench.json; grep -E "extra|head|strong" gpurun_out/bench.err
if [ -n "$GPU_ROUND_GLOO" ]; then
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --dist-backend gloo --steps 10 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || { echo "gloo rehearsal failed"; tail -30 gpurun_out/bench_gloo2.err; exit 1; }
  tail -c 1500 gpurun_out/bench_gloo2.json; grep -E "strong" gpurun_out/bench_gloo2.err
fi
