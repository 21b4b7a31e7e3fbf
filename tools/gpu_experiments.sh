#!/bin/bash
# Round-4 experiments, one GPU box, by name (each step bounded; the first failure ends the session):
#   done_event   back-to-back cost of a completion event per launch: lib vs variants/doneev
#                (tools/build_variant.sh doneev "-DMRT_DONE_EVENT")          -> profiles/round4_done_event_ab.txt
#   queue        rule vs per-XCD block-cyclic queue forms, times + fabric bytes (tools/pmc_configs.sh)
#                                                                            -> profiles/round4_queue_*.txt
#   wideq        quantized 64-B wide nodes vs exact on the hairball frames   -> profiles/round4_wideq_ab.txt
#   strong_launches   strong-scaling shards cut into 1..4 launches (bench --strong-min-launches)
#   strong_blocks     block size x balance of the strong-scaling shards (BLOCKS, BALANCE)
#   shard_sweep  the 8 shards under per-XCD queue variants, frame order     -> tools/strong_diag.py
#   order        live blocks first: dist block x balance x queue block      -> profiles/round4_order_sweep.txt
#   order2       live blocks first: ordering granularity x shared-queue share -> profiles/round4_order_sweep2.txt
#   shard_sched  live blocks first, 1024-ray blocks: the shards under slack / waves / tail / lane-group variants
#   shard_knobs  live blocks first, 1024-ray blocks: shared share / static rounds / refill threshold / tail lanes
#   shared_frame the shared-queue share on the 1 spp hairball frames and on ordered shards (0 / 2 / 5 %)
#   balance_final  the saved per-XCD schedule on ordered shards: dist block 512/1024/2048 x cyclic/balanced deal
#   shard_split  each ordered shard as 1 / 2 / 3 launches alternating over two streams (explicit schedule)
#   order_frame  one frame's batch in frame order vs live blocks first (tools/order_probe.py)
#   head_knobs   the headline batch under slack / lane-group / tail / stack variants of its saved schedule
#   head_knobs2  the headline's new schedule against its neighbours (lane groups 2/4, slack 4/6/8, waves 8/12/16)
#   small_xcd    per-XCD queues with smaller blocks on the 307 k-ray batches (vs their saved schedules)
#   deal_rot     ordered shards: block-cyclic deal vs the deal rotated by one rank per round
#   ao_knobs     Mori / Fairy AO under launch knobs the autotuner does not explore
#   timeline_shard  per-ray timeline of shard 0, live first vs frame order (variants/tailtl build)
# Round-5 experiments:
#   r5_guard     the unserved-queue sweep's cost: variants/noroot (this tree without the LDS root) vs the
#                round-4 kernel (variants/r4, tools/build_variant.sh r4 "" d775aa0), saved schedules
#   r5_root      the root visit from LDS: lib vs variants/noroot (tools/build_variant.sh noroot -DMRT_ROOT_LDS=0)
#   r5_hb640     hairball diffuse 640x480: global vs per-XCD queues x refill x waves x slack
#   r5_ao        Mori / Fairy AO: grid size and the frontier tail
#   r5_sort      the octant ray sort (cfg.ray_sort) of one-round static launches on the 307 k-ray batches
#   r5_order     projected eta(n) of the strong-scaling shards: live blocks first vs costly blocks first
#   (later round-5 A/Bs — the packet traversal, top levels in LDS, scheduler flags, XCD shares, ray prefetch —
#    were run from throwaway scripts against tools/build_variant.sh builds; their outputs are profiles/round5_*_ab.txt)
# Usage: gpurun -- 'bash tools/gpu_experiments.sh order order2'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
fail() { echo "$1 failed"; tail -20 "$2"; exit 1; }
Q8='"autotune":0,"num_queues":8,"fetch_threshold":48,"waves_per_cu":20'
for exp in "$@"; do
  case $exp in
    done_event)
      timeout -k 10 600 python -u tools/ab.py --rounds 7 --launches 30 --workload conference-ao-640x480 --workload mori-ao-640x480 \
        --workload bunny-primary-640x480 --workload bunny-primary-1024x768 --workload hairball-diffuse-1920x1080 \
        --variant 'lib:{"saved":1}' --variant 'lib/variants/doneev:{"saved":1}' --variant 'lib:{"autotune":0}' \
        --variant 'lib/variants/doneev:{"autotune":0}' > $O/ab_done.txt 2> $O/ab_done.err || fail ab $O/ab_done.err
      cat $O/ab_done.txt ;;
    queue)
      CFGS=('{"autotune":0}' "{$Q8,\"queue_shared\":10,\"queue_block\":16384}" "{$Q8,\"queue_shared\":5,\"queue_block\":4096}"
            "{$Q8,\"queue_shared\":5,\"queue_block\":8192}" "{$Q8,\"queue_shared\":10,\"queue_block\":65536}")
      V=""; for c in "${CFGS[@]}"; do V="$V --variant lib:$c"; done
      timeout -k 10 900 python -u tools/ab.py --rounds 5 --launches 20 --workload hairball-diffuse-1920x1080 --workload hairball-diffuse-640x480 \
        --workload bunny-primary-1024x768 --workload mori-ao-640x480 --workload conference-ao-640x480 $V > $O/ab_q.txt 2> $O/ab_q.err || fail ab $O/ab_q.err
      cat $O/ab_q.txt
      timeout -k 10 900 bash tools/pmc_configs.sh hairball-diffuse-1920x1080 "${CFGS[@]}" > $O/pmc_cfg.txt 2>&1 || fail pmc $O/pmc_cfg.txt
      cat $O/pmc_cfg.txt ;;
    wideq)
      X="$Q8,\"spec_slack\":6,\"queue_shared\":5,\"queue_block\":8192"
      timeout -k 10 500 python -u tools/ab.py --rounds 7 --launches 30 --workload hairball-diffuse-1920x1080 --workload hairball-diffuse-640x480 \
        --workload hairball-primary-1024x768 --variant "lib:{$X}" --variant "lib:{$X,\"wide\":2}" --variant 'lib:{"autotune":0}' \
        --variant 'lib:{"autotune":0,"wide":2}' > $O/ab_wideq.txt 2> $O/ab_wideq.err || fail ab $O/ab_wideq.err
      cat $O/ab_wideq.txt ;;
    strong_launches)
      for ML in 1 2 3 4; do
        timeout -k 10 300 python bench.py --no-extra --no-cpu --no-fast --no-explore --steps 20 --strong-min-launches $ML \
          --detail-out $O/strong_ml$ML.json > $O/strong_ml$ML.out 2> $O/strong_ml$ML.err || fail "ml $ML" $O/strong_ml$ML.err
        echo "min_launches $ML: $(grep strong $O/strong_ml$ML.err)"
      done ;;
    strong_blocks)
      for BAL in ${BALANCE:-1 0}; do for B in ${BLOCKS:-16384 4096 1024 256}; do
        T=b${B}_bal$BAL
        timeout -k 10 300 python bench.py --no-extra --no-cpu --no-fast --no-explore --steps 20 --strong-steps 20 --strong-block $B \
          --strong-balance $BAL --detail-out $O/strong_$T.json > $O/strong_$T.out 2> $O/strong_$T.err || fail $T $O/strong_$T.err
        python3 -c "
import json; d=json.load(open('$O/strong_$T.json'))['strong']
print('block $B balance $BAL T1', d['t1_ms'], 'one-stream', d.get('one_stream_ms'), {k: (v['eta'], [round(x,3) for x in v['shard_ms']]) for k, v in d['projected_from_one_gpu'].items()})"
      done; done ;;
    shard_sweep)
      EXTRA_SCHEDS="sh5b4096={$Q8,\"queue_shared\":5,\"queue_block\":4096};sh15b4096={$Q8,\"queue_shared\":15,\"queue_block\":4096};sh30b4096={$Q8,\"queue_shared\":30,\"queue_block\":4096};sh5b16384={$Q8,\"queue_shared\":5,\"queue_block\":16384}" \
      SCHEDS=sh5b4096,sh15b4096,sh30b4096,sh5b16384 ORDERS=fwd REPS=7 \
        timeout -k 10 600 python -u tools/strong_diag.py > $O/shard_sweep.txt 2> $O/shard_sweep.err || fail diag $O/shard_sweep.err
      cat $O/shard_sweep.txt ;;
    order)
      B="$Q8,\"spec_slack\":6,\"queue_shared\":5"
      timeout -k 10 400 python -u tools/ab.py --rounds 7 --launches 30 --workload hairball-diffuse-1920x1080 \
        --variant "lib:{$B,\"queue_block\":4096}" --variant "lib:{$B,\"queue_block\":8192}" --variant "lib:{$B,\"queue_block\":16384}" \
        > $O/ab_qblock.txt 2> $O/ab_qblock.err || fail ab $O/ab_qblock.err
      cat $O/ab_qblock.txt
      for BL in 1024 4096; do for BAL in 0 1; do
        EXTRA_SCHEDS="x4096={$B,\"queue_block\":4096};x8192={$B,\"queue_block\":8192};x16384={$B,\"queue_block\":16384}" \
        SCHEDS=x4096,x8192,x16384 ORDERS=fwd REPS=7 ORDER=1 BLOCK=$BL BALANCE=$BAL \
          timeout -k 10 300 python -u tools/strong_diag.py > $O/order_b${BL}_bal$BAL.txt 2> $O/order_b${BL}_bal$BAL.err || fail diag $O/order_b${BL}_bal$BAL.err
      done; done ;;
    order2)
      B="$Q8,\"spec_slack\":6"
      for BL in 256 1024; do
        EXTRA_SCHEDS="q8s5={$B,\"queue_block\":8192,\"queue_shared\":5};q8s10={$B,\"queue_block\":8192,\"queue_shared\":10};q8s20={$B,\"queue_block\":8192,\"queue_shared\":20};q16s10={$B,\"queue_block\":16384,\"queue_shared\":10}" \
        SCHEDS=q8s5,q8s10,q8s20,q16s10 ORDERS=fwd REPS=7 ORDER=1 BLOCK=$BL \
          timeout -k 10 300 python -u tools/strong_diag.py > $O/order2_b$BL.txt 2> $O/order2_b$BL.err || fail diag $O/order2_b$BL.err
      done ;;
    shard_sched)
      B="$Q8,\"queue_shared\":5"
      EXTRA_SCHEDS="s8k6={$B,\"queue_block\":8192,\"spec_slack\":6};s8k4={$B,\"queue_block\":8192,\"spec_slack\":4};s8k2={$B,\"queue_block\":8192};s16k6={$B,\"queue_block\":16384,\"spec_slack\":6};s16k4={$B,\"queue_block\":16384,\"spec_slack\":4};s8k6w16={$B,\"queue_block\":8192,\"spec_slack\":6,\"waves_per_cu\":16};s8k6t0={$B,\"queue_block\":8192,\"spec_slack\":6,\"tail_lanes\":0};s8k6lg={$B,\"queue_block\":8192,\"spec_slack\":6,\"lane_groups\":16}" \
      SCHEDS=s8k6,s8k4,s8k2,s16k6,s16k4,s8k6w16,s8k6t0,s8k6lg ORDERS=fwd REPS=7 ORDER=1 BLOCK=1024 \
        timeout -k 10 600 python -u tools/strong_diag.py > $O/shard_sched.txt 2> $O/shard_sched.err || fail diag $O/shard_sched.err ;;
    timeline_shard)
      X="$Q8,\"spec_slack\":6,\"queue_shared\":5,\"queue_block\":8192"
      for ORD in 1 0; do
        MRT_LIB_DIR=$PWD/gpu-ray-tracing_amd/lib/variants/tailtl EXTRA_SCHEDS="x8192={$X}" SCHEDS=x8192 BLOCK=1024 TIMELINE=1 ORDER=$ORD \
          timeout -k 10 300 python -u tools/strong_diag.py > $O/tlshard$ORD.txt 2> $O/tlshard$ORD.err || fail timeline $O/tlshard$ORD.err
        cat $O/tlshard$ORD.txt
      done ;;
    shard_knobs)
      B="$Q8,\"queue_block\":8192,\"spec_slack\":6"
      EXTRA_SCHEDS="base={$B,\"queue_shared\":5};sh2={$B,\"queue_shared\":2};sh0={$B,\"queue_shared\":0};sr2={$B,\"queue_shared\":5,\"static_rounds\":2};ft32={$B,\"queue_shared\":5,\"fetch_threshold\":32};ft56={$B,\"queue_shared\":5,\"fetch_threshold\":56};tl8={$B,\"queue_shared\":5,\"tail_lanes\":8}" \
      SCHEDS=base,sh2,sh0,sr2,ft32,ft56,tl8 ORDERS=fwd REPS=7 ORDER=1 BLOCK=1024 \
        timeout -k 10 600 python -u tools/strong_diag.py > $O/shard_knobs.txt 2> $O/shard_knobs.err || fail diag $O/shard_knobs.err ;;
    shared_frame)
      B="$Q8,\"spec_slack\":6"
      V=""
      for c in "{$B,\"queue_block\":8192,\"queue_shared\":5}" "{$B,\"queue_block\":8192,\"queue_shared\":2}" "{$B,\"queue_block\":8192,\"queue_shared\":0}" \
               "{$B,\"queue_block\":4096,\"queue_shared\":0}" "{$B,\"queue_block\":16384,\"queue_shared\":0}" "{$B,\"queue_block\":8192,\"queue_shared\":0,\"fetch_threshold\":56}"; do
        V="$V --variant lib:$c"
      done
      timeout -k 10 500 python -u tools/ab.py --rounds 7 --launches 30 --workload hairball-diffuse-1920x1080 --workload hairball-diffuse-640x480 $V \
        > $O/ab_shared.txt 2> $O/ab_shared.err || fail ab $O/ab_shared.err
      cat $O/ab_shared.txt
      B2="$B,\"queue_shared\":0"
      EXTRA_SCHEDS="s0b8={$B2,\"queue_block\":8192};s0b16={$B2,\"queue_block\":16384};s0b4={$B2,\"queue_block\":4096};s0b8f56={$B2,\"queue_block\":8192,\"fetch_threshold\":56}" \
      SCHEDS=s0b8,s0b16,s0b4,s0b8f56 ORDERS=fwd REPS=7 ORDER=1 BLOCK=1024 \
        timeout -k 10 600 python -u tools/strong_diag.py > $O/shard_shared0.txt 2> $O/shard_shared0.err || fail diag $O/shard_shared0.err ;;
    balance_final)
      X='"autotune":0,"num_queues":8,"fetch_threshold":56,"waves_per_cu":20,"spec_slack":6,"queue_block":8192,"queue_shared":0'
      for BL in 512 1024 2048; do for BAL in 0 1; do
        EXTRA_SCHEDS="c2={$X}" SCHEDS=c2 ORDERS=fwd REPS=9 ORDER=1 BLOCK=$BL BALANCE=$BAL \
          timeout -k 10 300 python -u tools/strong_diag.py > $O/bal_b${BL}_$BAL.txt 2> $O/bal_b${BL}_$BAL.err || fail diag $O/bal_b${BL}_$BAL.err
      done; done ;;
    shard_split)
      X='"autotune":0,"num_queues":8,"fetch_threshold":56,"waves_per_cu":20,"spec_slack":6,"queue_block":8192,"queue_shared":0'
      for SP in 1 2 3; do
        EXTRA_SCHEDS="c2={$X}" SCHEDS=c2 ORDERS=fwd REPS=9 ORDER=1 BLOCK=1024 SPLIT=$SP \
          timeout -k 10 300 python -u tools/strong_diag.py > $O/split_$SP.txt 2> $O/split_$SP.err || fail diag $O/split_$SP.err
      done ;;
    order_frame)
      X='{"autotune":0,"num_queues":8,"fetch_threshold":56,"waves_per_cu":20,"spec_slack":6,"queue_block":8192,"queue_shared":0}'
      for W in hairball-diffuse-1920x1080 hairball-diffuse-640x480 sponza-diffuse-640x480 conference-ao-640x480; do
        timeout -k 10 300 python -u tools/order_probe.py $W "$X" 256 1024 4096 >> $O/order_frame.txt 2>> $O/order_frame.err || fail probe $O/order_frame.err
        timeout -k 10 300 python -u tools/order_probe.py $W '{"autotune":0}' 1024 >> $O/order_frame.txt 2>> $O/order_frame.err || fail probe $O/order_frame.err
      done
      cat $O/order_frame.txt ;;
    head_knobs)
      V=""
      for c in '{"autotune":0,"waves_per_cu":8,"spec_slack":6}' '{"autotune":0,"waves_per_cu":8,"spec_slack":8}' \
               '{"autotune":0,"waves_per_cu":8,"spec_slack":10}' '{"autotune":0,"waves_per_cu":8,"spec_slack":14}' \
               '{"autotune":0,"waves_per_cu":8,"spec_slack":20}' '{"autotune":0,"waves_per_cu":8,"spec_slack":6,"lane_groups":2}' \
               '{"autotune":0,"waves_per_cu":8,"spec_slack":6,"tail_lanes":8}' '{"autotune":0,"waves_per_cu":8,"spec_slack":6,"lds_stack":8}' \
               '{"autotune":0,"waves_per_cu":12,"spec_slack":8}'; do
        V="$V --variant lib:$c"
      done
      timeout -k 10 600 python -u tools/ab.py --rounds 9 --launches 30 --workload bunny-primary-1024x768 --workload bunny-primary-640x480 $V \
        > $O/ab_head.txt 2> $O/ab_head.err || fail ab $O/ab_head.err
      cat $O/ab_head.txt ;;
    head_knobs2)
      V=""
      for c in '{"autotune":0,"waves_per_cu":8,"spec_slack":6,"lane_groups":2}' '{"autotune":0,"waves_per_cu":8,"spec_slack":6,"lane_groups":4}' \
               '{"autotune":0,"waves_per_cu":8,"spec_slack":4,"lane_groups":2}' '{"autotune":0,"waves_per_cu":8,"spec_slack":8,"lane_groups":2}' \
               '{"autotune":0,"waves_per_cu":12,"spec_slack":6,"lane_groups":2}' '{"autotune":0,"waves_per_cu":8,"spec_slack":6,"lane_groups":2,"tail_lanes":12}' \
               '{"autotune":0,"waves_per_cu":8,"spec_slack":6,"lane_groups":2,"static_rounds":1}' '{"autotune":0,"waves_per_cu":16,"spec_slack":6,"lane_groups":4}'; do
        V="$V --variant lib:$c"
      done
      timeout -k 10 600 python -u tools/ab.py --rounds 9 --launches 30 --workload bunny-primary-1024x768 --workload fairy-ao-640x480 --workload mori-ao-640x480 $V \
        > $O/ab_head2.txt 2> $O/ab_head2.err || fail ab $O/ab_head2.err
      cat $O/ab_head2.txt ;;
    small_xcd)
      V='--variant lib:{"saved":1}'
      for B in 1024 2048 4096; do for W in 12 20; do
        V="$V --variant lib:{\"autotune\":0,\"num_queues\":8,\"fetch_threshold\":56,\"waves_per_cu\":$W,\"spec_slack\":6,\"queue_block\":$B}"
      done; done
      timeout -k 10 600 python -u tools/ab.py --rounds 9 --launches 30 --workload hairball-diffuse-640x480 --workload hairball-primary-640x480 \
        --workload sponza-diffuse-640x480 $V > $O/ab_small_xcd.txt 2> $O/ab_small_xcd.err || fail ab $O/ab_small_xcd.err
      cat $O/ab_small_xcd.txt ;;
    deal_rot)
      X='"autotune":0,"num_queues":8,"fetch_threshold":56,"waves_per_cu":20,"spec_slack":6,"queue_block":8192,"queue_shared":0'
      for D in cyc rot; do
        EXTRA_SCHEDS="c2={$X}" SCHEDS=c2 ORDERS=fwd REPS=15 ORDER=1 BLOCK=1024 DEAL=$D \
          timeout -k 10 300 python -u tools/strong_diag.py > $O/deal_$D.txt 2> $O/deal_$D.err || fail diag $O/deal_$D.err
      done ;;
    ao_knobs)
      V=""
      for c in '{"autotune":0}' '{"autotune":0,"spec_slack":4}' '{"autotune":0,"tail_lanes":8}' '{"autotune":0,"tail_lanes":4}' \
               '{"autotune":0,"lane_groups":4}' '{"autotune":0,"lane_groups":2}' '{"autotune":0,"lds_stack":8}' \
               '{"autotune":0,"waves_per_cu":16}' '{"autotune":0,"waves_per_cu":16,"lane_groups":4}' '{"autotune":0,"spec_slack":8}'; do
        V="$V --variant lib:$c"
      done
      timeout -k 10 600 python -u tools/ab.py --rounds 7 --launches 30 --workload mori-ao-640x480 --workload fairy-ao-640x480 $V \
        > $O/ab_ao.txt 2> $O/ab_ao.err || fail ab $O/ab_ao.err
      cat $O/ab_ao.txt ;;
    r5_guard)
      timeout -k 10 600 python -u tools/ab.py --rounds 11 --launches 30 --workload hairball-diffuse-1920x1080 \
        --workload bunny-primary-1024x768 --workload hairball-diffuse-640x480 --workload conference-ao-640x480 \
        --variant 'lib/variants/noroot:{"saved":1}' --variant 'lib/variants/r4:{"saved":1}' > $O/ab_guard.txt 2> $O/ab_guard.err || fail ab $O/ab_guard.err
      cat $O/ab_guard.txt ;;
    r5_root)   # the root visit from LDS: this tree vs variants/noroot (-DMRT_ROOT_LDS=0), saved schedules
      timeout -k 10 600 python -u tools/ab.py --rounds 9 --launches 30 --workload bunny-primary-1024x768 --workload bunny-primary-640x480 \
        --workload conference-ao-640x480 --workload sponza-diffuse-640x480 --workload hairball-diffuse-640x480 \
        --workload hairball-diffuse-1920x1080 --workload mori-ao-640x480 --workload fairy-ao-640x480 \
        --variant 'lib:{"saved":1}' --variant 'lib/variants/noroot:{"saved":1}' > $O/ab_root.txt 2> $O/ab_root.err || fail ab $O/ab_root.err
      cat $O/ab_root.txt ;;
    r5_hb640)
      V='--variant lib:{"saved":1}'
      for W in 12 16; do for T in 40 48 56; do
        V="$V --variant lib:{\"autotune\":0,\"num_queues\":1,\"fetch_threshold\":$T,\"waves_per_cu\":$W}"
      done; done
      for B in 1024 4096; do for W in 12 16; do
        V="$V --variant lib:{\"autotune\":0,\"num_queues\":8,\"fetch_threshold\":48,\"waves_per_cu\":$W,\"queue_block\":$B}"
      done; done
      V="$V --variant lib:{\"autotune\":0,\"num_queues\":1,\"fetch_threshold\":48,\"waves_per_cu\":12,\"spec_slack\":4}"
      V="$V --variant lib:{\"autotune\":0,\"num_queues\":1,\"fetch_threshold\":48,\"waves_per_cu\":12,\"tail_lanes\":8}"
      V="$V --variant lib:{\"autotune\":0,\"num_queues\":1,\"fetch_threshold\":48,\"waves_per_cu\":12,\"static_rounds\":2}"
      timeout -k 10 600 python -u tools/ab.py --rounds 9 --launches 30 --workload hairball-diffuse-640x480 $V \
        > $O/ab_hb640.txt 2> $O/ab_hb640.err || fail ab $O/ab_hb640.err
      cat $O/ab_hb640.txt ;;
    r5_ao)
      V='--variant lib:{"saved":1}'
      for W in 4 6 8 12 16 20 24 32; do V="$V --variant lib:{\"autotune\":0,\"waves_per_cu\":$W}"; done
      V="$V --variant lib:{\"autotune\":0,\"tail_lanes\":0}"
      timeout -k 10 600 python -u tools/ab.py --rounds 7 --launches 30 --workload mori-ao-640x480 --workload fairy-ao-640x480 $V \
        > $O/ab_ao5.txt 2> $O/ab_ao5.err || fail ab $O/ab_ao5.err
      cat $O/ab_ao5.txt ;;
    r5_order)   # projected eta(2/4/8) with the shard blocks live-first (1) vs cost-first (2), three runs each
      for run in 1 2 3; do for OR in 1 2; do
        timeout -k 10 400 python bench.py --no-extra --no-cpu --no-explore --no-fast --steps 5 --strong-order $OR \
          --detail-out $O/order${OR}_$run.json > $O/order${OR}_$run.line 2> $O/order${OR}_$run.err || fail bench $O/order${OR}_$run.err
        python3 -c "
import json; d=json.load(open('$O/order${OR}_$run.json'))['strong']
print('order $OR run $run T1', d['t1_ms'], {k: (v['eta'], max(v['shard_ms'])) for k, v in d['projected_from_one_gpu'].items()})" | tee -a $O/order_r5.txt
      done; done ;;
    r5_sort)   # the octant ray sort of one-round static launches
      V='--variant lib:{"saved":1} --variant lib:{"autotune":0} --variant lib:{"autotune":0,"ray_sort":1}'
      V="$V --variant lib:{\"autotune\":0,\"ray_sort\":1,\"tail_lanes\":0} --variant lib:{\"autotune\":0,\"ray_sort\":1,\"spec_slack\":4}"
      timeout -k 10 600 python -u tools/ab.py --rounds 7 --launches 30 --workload mori-ao-640x480 --workload fairy-ao-640x480 \
        --workload conference-ao-640x480 --workload sponza-ao-640x480 --workload san-ao-640x480 --workload bunny-primary-640x480 \
        --workload sponza-diffuse-640x480 --workload hairball-diffuse-640x480 --workload mori-diffuse-640x480 $V \
        > $O/ab_sort.txt 2> $O/ab_sort.err || fail ab $O/ab_sort.err
      cat $O/ab_sort.txt ;;
    r5_regs)   # this tree (ray-sort code present, off) vs the tree before it (variants/presort) vs round 4
      timeout -k 10 600 python -u tools/ab.py --rounds 9 --launches 30 --workload hairball-diffuse-640x480 \
        --workload hairball-diffuse-1920x1080 --workload bunny-primary-1024x768 --workload bunny-primary-640x480 \
        --workload conference-ao-640x480 --workload sponza-diffuse-640x480 --workload mori-ao-640x480 \
        --variant 'lib:{"saved":1}' --variant 'lib/variants/presort:{"saved":1}' --variant 'lib/variants/sort0:{"saved":1}' \
        > $O/ab_regs.txt 2> $O/ab_regs.err || fail ab $O/ab_regs.err
      cat $O/ab_regs.txt ;;
    r5_probe)   # which part of the (disabled) ray-sort block speeds the kernel up: its LDS, or a barrier
      timeout -k 10 600 python -u tools/ab.py --rounds 9 --launches 30 --workload hairball-diffuse-1920x1080 \
        --workload bunny-primary-1024x768 --workload sponza-diffuse-640x480 --workload hairball-diffuse-640x480 \
        --variant 'lib:{"saved":1}' --variant 'lib/variants/sort0:{"saved":1}' --variant 'lib/variants/ldspad:{"saved":1}' \
        --variant 'lib/variants/dbar:{"saved":1}' > $O/ab_probe.txt 2> $O/ab_probe.err || fail ab $O/ab_probe.err
      cat $O/ab_probe.txt ;;
    r5_nops)   # is the dead-code speed-up code placement? sort0 shifted by 1/2/4/8 s_nop
      timeout -k 10 600 python -u tools/ab.py --rounds 9 --launches 30 --workload hairball-diffuse-640x480 \
        --workload bunny-primary-1024x768 --workload hairball-diffuse-1920x1080 \
        --variant 'lib:{"saved":1}' --variant 'lib/variants/sort0:{"saved":1}' --variant 'lib/variants/nop1:{"saved":1}' \
        --variant 'lib/variants/nop2:{"saved":1}' --variant 'lib/variants/nop4:{"saved":1}' --variant 'lib/variants/nop8:{"saved":1}' \
        --variant 'lib/variants/al64:{"saved":1}' --variant 'lib/variants/cur_al64:{"saved":1}' \
        > $O/ab_nops.txt 2> $O/ab_nops.err || fail ab $O/ab_nops.err
      cat $O/ab_nops.txt ;;
    r5_slack)   # any-hit batches: turn to the postponed leaves earlier (spec_slack 8 .. 63 = as soon as one lane has one)
      V='--variant lib:{"autotune":0}'
      for K in 8 16 32 48 63; do V="$V --variant lib:{\"autotune\":0,\"spec_slack\":$K}"; done
      timeout -k 10 600 python -u tools/ab.py --rounds 7 --launches 30 --workload mori-ao-640x480 --workload fairy-ao-640x480 \
        --workload conference-ao-640x480 --workload sponza-ao-640x480 $V > $O/ab_slack.txt 2> $O/ab_slack.err || fail ab $O/ab_slack.err
      cat $O/ab_slack.txt ;;
    r5_steal)   # end-of-batch queue stealing (cfg.queue_steal): its code's cost (off, vs variants/presteal) and its effect
                # (the knob was removed after this run: check out aff58af to repeat it)
      X='"autotune":0,"num_queues":8,"fetch_threshold":56,"waves_per_cu":20,"spec_slack":6,"queue_block":8192'
      Y='"autotune":0,"num_queues":8,"fetch_threshold":48,"waves_per_cu":12'
      timeout -k 10 600 python -u tools/ab.py --rounds 9 --launches 30 --workload hairball-diffuse-1920x1080 \
        --workload hairball-diffuse-640x480 --workload bunny-primary-1024x768 --workload sponza-diffuse-640x480 \
        --variant 'lib:{"saved":1}' --variant 'lib/variants/presteal:{"saved":1}' \
        --variant "lib:{$X}" --variant "lib:{$X,\"queue_steal\":1}" \
        --variant "lib:{$Y,\"queue_block\":1024}" --variant "lib:{$Y,\"queue_block\":1024,\"queue_steal\":1}" \
        --variant "lib:{$Y,\"queue_block\":4096,\"queue_steal\":1}" \
        > $O/ab_steal.txt 2> $O/ab_steal.err || fail ab $O/ab_steal.err
      cat $O/ab_steal.txt ;;
    r5_balance)   # projected eta(n): blocks dealt cyclically (0) vs by the next frame's cost (2), live-first order, three runs each
      for run in 1 2 3; do for BAL in 0 2; do
        timeout -k 10 400 python bench.py --no-extra --no-cpu --no-explore --no-fast --steps 5 --strong-balance $BAL \
          --detail-out $O/bal${BAL}_$run.json > $O/bal${BAL}_$run.line 2> $O/bal${BAL}_$run.err || fail bench $O/bal${BAL}_$run.err
        python3 -c "
import json; d=json.load(open('$O/bal${BAL}_$run.json'))['strong']
print('balance $BAL run $run T1', d['t1_ms'], {k: (v['eta'], max(v['shard_ms']), min(v['shard_ms'])) for k, v in d['projected_from_one_gpu'].items()})" | tee -a $O/balance_r5.txt
      done; done ;;
    r5_head)   # the headline batch around its saved schedule (static rounds, 8 waves/CU, 2 lane groups, slack 6)
      V='--variant lib:{"saved":1}'
      for c in '"spec_slack":8' '"spec_slack":10' '"tail_lanes":8' '"tail_lanes":0' '"lds_stack":8' '"lane_groups":4' \
               '"waves_per_cu":12' '"waves_per_cu":4' '"lane_groups":2,"spec_slack":4' '"static_rounds":1,"spec_slack":7'; do
        V="$V --variant lib:{\"autotune\":0,\"waves_per_cu\":8,\"lane_groups\":2,\"spec_slack\":6,$c}"
      done
      timeout -k 10 600 python -u tools/ab.py --rounds 9 --launches 30 --workload bunny-primary-1024x768 $V \
        > $O/ab_head5.txt 2> $O/ab_head5.err || fail ab $O/ab_head5.err
      cat $O/ab_head5.txt ;;
    *) echo "unknown experiment $exp"; exit 2 ;;
  esac
done
