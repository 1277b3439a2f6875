#!/bin/bash
# round 4 end (after the small-kernel / optimizer work), measurement pass: PMC traffic + MFMA passes, kernel
# trace + step timeline, DP trace, the default bench line into profiles/r04_*, then the configs[4] (dual,
# base 96, 2048^2) bench line.  The conv kernels' SQ attribution and stamps are unchanged since
# tools/gpu_r4_final_b.sh (profiles/r04_sq_layers_final.txt, r04_conv_stamps.txt).
set -u
TAG=${TAG:-r4g} R=r04 bash tools/gpu_round_final.sh || exit $?
timeout -k 10 600 python bench.py --dual --base 96 --size 2048 --batch 2 --steps 5 --warmup 2 --no-cpu-baseline \
  --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/bench_dual.log 2>&1 || { echo "dual bench failed"; tail -5 gpurun_out/bench_dual.log; exit 1; }
grep "^{" gpurun_out/bench_dual.log | tail -1 > profiles/r04_bench_dual_cfg5.json
echo done
