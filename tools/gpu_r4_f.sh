#!/bin/bash
# round 4: conv B1 (weights staged by buffer_load ... lds: no staging registers, no ds_write, one round trip
# less per K-chunk) and head H3 (head_out32 packed BN+ReLU into the 1x1's bf16 fragments; head_bwd1 channel
# sums as MFMAs over pixels) vs W1: parity with the variant libraries, per-layer conv_bench, head kernels, bench
set -u
EUNET_LIB=abl/libh3.so TAG=head_h3 TLIM=400 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "head" || exit $?
EUNET_LIB=abl/libb1.so TAG=conv_b1 TLIM=500 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "conv" || exit $?
EUNET_LIB=abl/libb1h3.so TAG=model_b1h3 TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_model.py tests/test_gpu_dual.py || exit $?
LIBS="abl/libw1.so abl/libb1.so" ROUNDS=2 bash tools/gpu_cb_libs.sh || exit $?
LIBS="abl/libh3.so" REPS=10 TAG=h3 bash tools/gpu_head_libs.sh || exit $?
for L in abl/libw1.so abl/libb1h3.so abl/libw1.so abl/libb1h3.so; do
  EUNET_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/r4f_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4f_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4f_bench.log | head -1) $(grep -o '"encoder_fwd": {"achieved": [0-9.]*, "frac": [0-9.]*' gpurun_out/r4f_bench.log)"
done
