#!/bin/bash
# tools/conv_bench.py (per-layer fwd / dgrad / wgrad, standalone) for each library in LIBS (alternating)
set -u
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-2}); do
  for L in $LIBS; do
    timeout -k 10 150 env EUNET_LIB=$L python tools/conv_bench.py --transform --reps 10 > gpurun_out/cb_libs.log 2>&1 || { echo "cb failed $L"; tail -3 gpurun_out/cb_libs.log; exit 1; }
    echo "$L $(grep summary gpurun_out/cb_libs.log)"
  done
done
