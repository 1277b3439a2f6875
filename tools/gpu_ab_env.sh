#!/bin/bash
# Generic same-box A/B of the default bench: alternating runs with env assignments A and B
# (e.g. A="EUNET_FUSE_SMALL_BNBWD=1" B="EUNET_FUSE_SMALL_BNBWD=0"), ROUNDS pairs, 30 timed steps each.
set -u
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-3}); do
  for tag in A B; do
    assign=${!tag}
    env $assign timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg --no-dual-leg ${BENCH_ARGS:-} \
      > gpurun_out/ab_env.log 2>&1 || { echo "bench failed ($assign)"; tail -3 gpurun_out/ab_env.log; exit 1; }
    grep "^{" gpurun_out/ab_env.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag [$assign]', d['value'], d['ms_per_step'])"
  done
done
