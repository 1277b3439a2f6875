#!/bin/bash
# round 4: head H1 (head_out32 packed BN+ReLU into the 1x1's bf16 fragments; head_gh b1 gradient from a ones
# column of the W1-gradient MFMAs, pixel mask on border tiles only) and H2 (H1 + head_bwd1's channel sums as
# MFMAs over pixels): head parity with each library, per-kernel head times, bench
set -u
for L in abl/libh2.so abl/libh1.so; do
  n=$(basename $L .so)
  EUNET_LIB=$L TAG=head_$n TLIM=400 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "head" || exit $?
done
EUNET_LIB=abl/libh2.so TAG=model_h2 TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_model.py tests/test_gpu_dual.py || exit $?
LIBS="abl/libh1.so abl/libh2.so" REPS=10 TAG=h12 bash tools/gpu_head_libs.sh || exit $?
for L in "" abl/libh2.so "" abl/libh2.so; do
  EUNET_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/r4e_bench.log 2>&1 || exit $?
  echo "bench lib=${L:-intree} $(grep -o '"value": [0-9.]*' gpurun_out/r4e_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4e_bench.log | head -1)"
done
