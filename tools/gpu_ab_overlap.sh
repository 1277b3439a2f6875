#!/bin/bash
# A/B of the side-stream weight-gradient overlap on one box: alternating runs, 20 timed steps each.
set -u
mkdir -p gpurun_out
for i in 1 2 3 4; do
  for mode in "" "--no-overlap"; do
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --dice-size 0 $mode \
      > gpurun_out/ab_ovl.log 2>&1 || { echo "bench failed ($mode)"; tail -3 gpurun_out/ab_ovl.log; exit 1; }
    grep "^{" gpurun_out/ab_ovl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('${mode:-overlap}', d['value'], d['ms_per_step'])"
  done
done
