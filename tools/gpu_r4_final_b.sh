#!/bin/bash
# round 4 end, part B: the measurement pass (PMC traffic + MFMA busy, kernel trace + step timeline, DP trace,
# the default bench line) into profiles/r04_*, then the per-layer SQ attribution of the final conv kernels
# and the configs[4] (dual-branch, base 96, 2048^2) bench line
set -u
TAG=${TAG:-r4f} R=r04 bash tools/gpu_round_final.sh || exit $?
TAG=sqf bash tools/gpu_sq_layers.sh > gpurun_out/sqf_run.log 2>&1 || { echo "sq failed"; tail -5 gpurun_out/sqf_run.log; exit 1; }
{ echo "# tools/gpu_sq_layers.sh at round-4 end (final kernels: weight / plain-dgrad halo LDS-DMA, wgrad buffer-DMA staging):"
  echo "# two rocprofv3 --pmc passes over tools/conv_bench.py --reps 1, joined per dispatch (tools/sq_layers.py)"
  cat gpurun_out/pmc_sqf_summary.txt; } > profiles/r04_sq_layers_final.txt
timeout -k 10 600 python bench.py --dual --base 96 --size 2048 --batch 2 --steps 5 --warmup 2 --no-cpu-baseline \
  --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/bench_dual.log 2>&1 || { echo "dual bench failed"; tail -5 gpurun_out/bench_dual.log; exit 1; }
grep "^{" gpurun_out/bench_dual.log | tail -1 > profiles/r04_bench_dual_cfg5.json
echo done
EUNET_LIB=abl/libstamp.so timeout -k 10 300 python tools/conv_stamps.py > gpurun_out/conv_stamps_final.txt 2>&1 || { echo "conv stamps failed"; exit 1; }
EUNET_LIB=abl/libstamp.so timeout -k 10 200 python tools/head_stamps.py > gpurun_out/head_stamps_final.txt 2>&1 || { echo "head stamps failed"; tail -3 gpurun_out/head_stamps_final.txt; exit 1; }
grep -h "layer\|kernel" gpurun_out/conv_stamps_final.txt gpurun_out/head_stamps_final.txt | tail -30
