#!/bin/bash
# Round 5: reproduce the driver's fp32 configs[1] leg (BENCH_r04: 46 img/s) with per-step spreads
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 > gpurun_out/r5a_drv.log 2>&1 || { echo fail1; tail -20 gpurun_out/r5a_drv.log; exit 1; }
timeout -k 10 400 python -u bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline --dice-size 0 > gpurun_out/r5a_def.log 2>&1 || { echo fail2; tail -20 gpurun_out/r5a_def.log; exit 1; }
timeout -k 10 300 python -u bench.py --dtype fp32 --size 512 --batch 8 --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 > gpurun_out/r5a_fp32.log 2>&1 || { echo fail3; tail -20 gpurun_out/r5a_fp32.log; exit 1; }
echo done
