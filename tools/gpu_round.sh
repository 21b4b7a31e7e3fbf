#!/bin/bash
# One GPU-box session as a list of steps, run in order; the first failing step ends the session
# and every GPU step runs under a time limit of its own. Steps:
#   test[=EXPR]     pytest -m gpu (with -k EXPR)                   -> gpurun_out/pytest_gpu.log
#   smoke           __graft_entry__.smoke()                        -> gpurun_out/smoke.log
#   bench[=ARGS]    bench.py ARGS (commas become spaces)           -> gpurun_out/bench.json, bench_detail.json
#   gloo            the N=2 flow, two gloo ranks on the one GPU, started by bench.py itself -> gpurun_out/bench_gloo2.json
#   gloorun         the same under torch.distributed.run           -> gpurun_out/bench_gloorun2.json
#   tune            steady-state schedules of the bench workloads  -> gpurun_out/tuned_schedules.json
#   profile=TAG     rocprofv3 kernel stats + PMC summaries of the bench workloads (PROF_WL overrides the list)
#                                                                  -> gpurun_out/profiles/TAG_*
#   readme          every README cell tuned, measured and checked  -> gpurun_out/readme_table.md
#   pipe=W          vector-memory / VALU pipeline counters of workload W (4 PMC passes) -> gpurun_out/pipe_W.txt
#   timeline=W      per-ray start / tail entry / end of workload W (MRT_TAIL_TIMELINE variant library)
# Usage: bash tools/gpu_round.sh test smoke bench      (gpurun -- 'bash tools/gpu_round.sh ...')
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
BENCH_WL="bunny-primary-1024x768 bunny-primary-640x480 conference-ao-640x480 sponza-diffuse-640x480 sponza-diffuse2-640x480 hairball-diffuse-640x480 hairball-diffuse-1920x1080 mori-ao-640x480 fairy-ao-640x480"
fail() { echo "$1 failed"; tail -30 "$2"; exit 1; }
for step in "$@"; do
  arg=""; [[ $step == *=* ]] && { arg=${step#*=}; step=${step%%=*}; }
  case $step in
    test)
      K=(); [ -n "$arg" ] && K=(-k "$arg")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider "${K[@]}" \
        > $O/pytest_gpu.log 2>&1 || { grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; fail pytest $O/pytest_gpu.log; }
      tail -1 $O/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke $O/smoke.log
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py ${arg//,/ } --detail-out $O/bench_detail.json > $O/bench.json 2> $O/bench.err || fail bench $O/bench.err
      grep -E "\[(head|extra|strong|line)\]" $O/bench.err ;;
    gloo)   # bench.py starts its two ranks itself (no launcher), as `python bench.py --gpus N` would
      timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --steps 10 --detail-out $O/bench_gloo2_detail.json \
        > $O/bench_gloo2.json 2> $O/bench_gloo2.err || fail "gloo rehearsal" $O/bench_gloo2.err
      grep -E "\[(head|strong|launch)\]" $O/bench_gloo2.err ;;
    gloorun)   # the same under torch.distributed.run (the driver's N>1 launch)
      timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
        bench.py --gpus 2 --dist-backend gloo --steps 10 --detail-out $O/bench_gloorun2_detail.json > $O/bench_gloorun2.json 2> $O/bench_gloorun2.err \
        || fail "gloo rehearsal (torchrun)" $O/bench_gloorun2.err
      grep -E "\[(head|strong)\]" $O/bench_gloorun2.err ;;
    tune)
      rm -f $O/tuned_schedules.json
      W=""; for w in $BENCH_WL; do [ $w = hairball-diffuse-1920x1080 ] || W="$W --workload $w"; done
      timeout -k 10 720 python -u tools/tune_db.py $W ${TUNE_ARGS} --out $O/tuned_schedules.json > $O/tune_db.txt 2> $O/tune_db.err || fail tune_db $O/tune_db.err
      timeout -k 10 240 python -u tools/tune_db.py --workload hairball-diffuse-1920x1080 --margin 0.015 ${TUNE_ARGS} --out $O/tuned_schedules.json \
        >> $O/tune_db.txt 2>> $O/tune_db.err || fail "tune hairball" $O/tune_db.err
      timeout -k 10 180 python -u tools/tune_db.py --workload bunny-primary-1024x768 --fast-rcp ${TUNE_ARGS} --out $O/tuned_schedules.json \
        >> $O/tune_db.txt 2>> $O/tune_db.err || fail "tune fast" $O/tune_db.err
      cut -c1-300 $O/tune_db.txt ;;
    profile)
      timeout -k 10 1150 bash tools/profile_all.sh ${arg:-round} ${PROF_WL:-$BENCH_WL fast:bunny-primary-1024x768} || exit 1
      ls $O/profiles ;;
    readme)   # every README cell on the package's saved schedules (no per-cell locks — the
              # table reports what a user of the shipped table gets): the README cells' BVHs tuned into a copy of
              # the package table (cells of one BVH and batch size share one entry, the last tuned), then measured
      cp gpu-ray-tracing_amd/mrt/tuned_schedules.json $O/tuned_schedules_all.json
      W=$(python3 -c "import sys; sys.path.insert(0,'tools'); import readme_table as r; print(' '.join('--workload '+c[0] for c in r.CELLS))")
      timeout -k 10 900 python -u tools/tune_db.py $W --rounds 2 --launches 10 --out $O/tuned_schedules_all.json \
        > $O/tune_db_readme.txt 2> $O/tune_db_readme.err || fail "tune readme" $O/tune_db_readme.err
      timeout -k 10 900 python -u tools/readme_table.py --tune-db $O/tuned_schedules_all.json \
        > $O/readme_table.log 2>&1 \
        || fail "readme table" $O/readme_table.log
      cat $O/readme_table.md ;;
    pipe)
      P="GRBM_GUI_ACTIVE TA_BUSY_avr TA_BUFFER_READ_WAVEFRONTS_sum;TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_COUNT TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum"
      P="$P;SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS"
      P="$P;SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_ACTIVE_INST_VMEM TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
      timeout -k 10 900 bash tools/pmc_pipe.sh $arg $O/pipe_$arg "$P" > $O/pipe_$arg.log 2>&1 || fail "pipe $arg" $O/pipe_$arg.log
      python3 tools/pipe_summary.py $O/pipe_$arg > $O/pipe_$arg.txt && tail -12 $O/pipe_$arg.txt ;;
    tlb)   # address translation (UTCL1 hits/misses, UTCL2 busy) + L1->L2 requests of workload W (3 PMC passes)
      P="TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
      P="$P;TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_STALL_LFIFO_NO_RES_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum GRBM_GUI_ACTIVE"
      P="$P;TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
      timeout -k 10 900 bash tools/pmc_pipe.sh $arg $O/tlb_$arg "$P" > $O/tlb_$arg.log 2>&1 || fail "tlb $arg" $O/tlb_$arg.log
      python3 tools/pipe_summary.py $O/tlb_$arg > $O/tlb_$arg.txt && tail -14 $O/tlb_$arg.txt ;;
    timeline)
      MRT_LIB_DIR=$PWD/gpu-ray-tracing_amd/lib/variants/tailtl timeout -k 10 300 python -u tools/tail_timeline.py $arg \
        '{"tail_lanes": 0, "autotune": 0}' '{"tail_lanes": 16, "autotune": 0}' >> $O/tail_tl.txt 2>> $O/tail_tl.err || fail timeline $O/tail_tl.err
      cut -c1-400 $O/tail_tl.txt ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
