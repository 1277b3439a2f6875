#!/bin/bash
# round 4: PRY (plain dgrad: the fused BN-backward reduction's first-pass y loaded before the last K-chunk's
# MFMAs) and PFPRY (+ forward: next K-chunk's first halo half and BN constants loaded before the current
# chunk's MFMAs) vs the in-tree build (abl/libcur.so): parity, conv_bench, bench
set -u
EUNET_LIB=abl/libpfpry.so TAG=conv_pf TLIM=500 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "conv or dgrad" || exit $?
EUNET_LIB=abl/libpfpry.so TAG=model_pf TLIM=700 bash tools/gpu_run_tests.sh tests/test_gpu_model.py tests/test_gpu_dual.py || exit $?
LIBS="abl/libcur.so abl/libpry.so abl/libpfpry.so" ROUNDS=2 bash tools/gpu_cb_libs.sh || exit $?
for L in abl/libcur.so abl/libpfpry.so abl/libpry.so abl/libcur.so abl/libpfpry.so abl/libpry.so; do
  EUNET_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/r4l_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4l_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4l_bench.log | head -1) $(grep -o '"encoder_fwd": {"achieved": [0-9.]*, "frac": [0-9.]*' gpurun_out/r4l_bench.log)"
done
