#!/bin/bash
# A/B: register budget / occupancy variants (profiles/round1_tuning.md).
AB_WORKLOADS='bunny-primary-1024x768 bunny-primary-640x480 sponza-diffuse-640x480 conference-ao-640x480 hairball-diffuse-640x480' \
bash tools/ab_round.sh --variant 'lib:{}' --variant 'lib/variants/w6:{}' --variant 'lib/variants/nopk:{}' \
  --variant 'lib/variants/nopkw7:{}' --variant 'lib/variants/nopkw8:{"waves_per_cu":32}' --variant 'lib/variants/nopk:{"waves_per_cu":24}'
