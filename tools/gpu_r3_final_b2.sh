#!/bin/bash
# Round 3 final (1/3): all GPU tests, steady-state tuning of the bench workloads (every schedule x modifier;
# the 2 M-ray hairball batch with a 1.5 % margin; the headline's fast-reciprocal variant too), the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log | head; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
rm -f gpurun_out/tuned_schedules.json
W="--workload bunny-primary-1024x768 --workload bunny-primary-640x480 --workload conference-ao-640x480 --workload sponza-diffuse-640x480 --workload sponza-diffuse2-640x480 --workload hairball-diffuse-640x480"
timeout -k 10 900 python -u tools/tune_db.py $W --out gpurun_out/tuned_schedules.json > gpurun_out/tune_db.txt 2> gpurun_out/tune_db.err || { echo "tune_db failed"; tail -20 gpurun_out/tune_db.err; exit 1; }
timeout -k 10 300 python -u tools/tune_db.py --workload hairball-diffuse-1920x1080 --margin 0.015 --out gpurun_out/tuned_schedules.json >> gpurun_out/tune_db.txt 2>> gpurun_out/tune_db.err || { echo "tune hb failed"; tail gpurun_out/tune_db.err; exit 1; }
timeout -k 10 300 python -u tools/tune_db.py --workload bunny-primary-1024x768 --fast-rcp --out gpurun_out/tuned_schedules.json >> gpurun_out/tune_db.txt 2>> gpurun_out/tune_db.err || { echo "tune fast failed"; tail gpurun_out/tune_db.err; exit 1; }
cut -c1-500 gpurun_out/tune_db.txt
timeout -k 10 400 python bench.py --tune-db gpurun_out/tuned_schedules.json > gpurun_out/bench_t4.json 2> gpurun_out/bench_t4.err || { echo "bench failed"; tail -30 gpurun_out/bench_t4.err; exit 1; }
grep -E "extra|head|strong" gpurun_out/bench_t4.err
