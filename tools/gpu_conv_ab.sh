#!/bin/bash
# conv op tests under each library in LIBS, then tools/conv_bench.py (per-layer fwd / dgrad / wgrad) per library
set -u
mkdir -p gpurun_out
for L in $LIBS; do
  t=$(basename $L .so)
  EUNET_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -k "conv3x3" --timeout 200 --timeout-method thread > gpurun_out/cab_$t.log 2>&1
  rc=$?; echo "$t tests rc=$rc $(tail -1 gpurun_out/cab_$t.log)"; [ $rc -gt 1 ] && exit $rc
done
for i in $(seq 1 ${ROUNDS:-1}); do
  for L in $LIBS; do
    t=$(basename $L .so)
    EUNET_LIB=$L timeout -k 10 150 python tools/conv_bench.py --transform --reps 10 ${CB_ARGS:-} > gpurun_out/cb_$t.log 2>&1 || { echo "cb failed $L"; tail -3 gpurun_out/cb_$t.log; exit 1; }
    echo "$t $(grep summary gpurun_out/cb_$t.log)"
  done
done
