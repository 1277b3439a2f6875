#!/bin/bash
# round 4: conv E3 (single v_cvt_pk_bf16_f32 conversions, compile-time store rows) and W1 (wgrad staging
# by buffer LDS-DMA with per-tile scalar offsets): correctness of the in-tree build (W1) over every kernel
# using Vec16 pack, A/B E2 / E3 / W1, bench
set -u
TAG=ops TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py || exit $?
TAG=model TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_model.py tests/test_gpu_dual.py || exit $?
TAG=img TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_imgproc.py tests/test_gpu_data.py || exit $?
LIBS="abl/libe2.so abl/libe3.so abl/libw1.so" ROUNDS=2 bash tools/gpu_cb_libs.sh || exit $?
for L in abl/libe2.so abl/libe3.so abl/libw1.so abl/libe2.so abl/libe3.so abl/libw1.so; do
  EUNET_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/r4d_bench.log 2>&1 || exit $?
  echo "bench lib=${L:-new} $(grep -o '"value": [0-9.]*' gpurun_out/r4d_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4d_bench.log | head -1) $(grep -o '"encoder_fwd": {"achieved": [0-9.]*, "frac": [0-9.]*' gpurun_out/r4d_bench.log)"
done
