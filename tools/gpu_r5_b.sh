#!/bin/bash
# Round 5: the driver's exact bench command, twice, with the per-step spreads now in every leg
set -u
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5b_drv$i.log 2>&1 || { echo fail$i; tail -20 gpurun_out/r5b_drv$i.log; exit 1; }
done
echo done
