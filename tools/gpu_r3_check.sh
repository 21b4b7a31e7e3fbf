#!/bin/bash
# GPU tests, an A/B of the round-2 library against this one (no-tail and tail kernels), then the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log | head; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
V="--variant lib/variants/r2:{\"autotune\":0} --variant lib:{\"autotune\":0} --variant lib:{\"autotune\":0,\"tail_lanes\":16}"
timeout -k 10 600 python -u tools/ab.py --rounds 7 --launches 30 --workload conference-ao-640x480 --workload bunny-primary-1024x768 \
   --workload bunny-primary-640x480 --workload sponza-diffuse-640x480 --workload hairball-diffuse-640x480 $V > gpurun_out/ab_final.txt 2> gpurun_out/ab_final.err || { echo "ab failed"; tail -20 gpurun_out/ab_final.err; exit 1; }
cat gpurun_out/ab_final.txt
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { echo "bench failed"; tail -30 gpurun_out/bench_final.err; exit 1; }
grep -E "extra|head|strong" gpurun_out/bench_final.err
