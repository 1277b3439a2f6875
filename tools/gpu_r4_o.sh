#!/bin/bash
# round 4: HIP stream priorities -- the step's stream high (weight-gradient side stream normal), the side
# stream high, neither -- alternating bench runs on one box
set -u
B="--steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg"
for M in none main side none main side none main side; do
  timeout -k 10 300 python tools/bench_prio.py $M -- $B > gpurun_out/r4o_bench.log 2>&1 || exit $?
  echo "bench prio=$M $(grep -o '"value": [0-9.]*' gpurun_out/r4o_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4o_bench.log | head -1) $(grep -o 'priority range.*' gpurun_out/r4o_bench.log | head -1)"
done
