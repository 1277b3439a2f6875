#!/bin/bash
# Round 4: per-layer SQ stall attribution (conv) + per-kernel (head), then a short bench for the box.
set -u
TAG=sql bash tools/gpu_sq_layers.sh || exit $?
TAG=sqh SQ_BY_KERNEL=1 PROG="python tools/head_bench.py --reps 3" bash tools/gpu_sq_layers.sh || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg \
  > gpurun_out/r4_bench0.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/r4_bench0.log; exit $rc
