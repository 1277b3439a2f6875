#!/bin/bash
# round 4: conv P3 (forward halo pixel-major in LDS) and A3 (P3 + the halo by buffer_load ... lds for the
# untransformed forwards and the plain data gradients: 16 pixels' 64 contiguous bytes per wave-instruction),
# head_gh variants (gu1: the two rows of a pair unrolled, 3 blocks / CU; gu2: unrolled, 2 blocks / CU, 512-block
# grid; go2: 2 blocks / CU only) vs B1+H3: parity with each library, conv_bench, head kernels, bench
set -u
EUNET_LIB=abl/liba3h3.so TAG=conv_a3 TLIM=500 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "conv or dgrad" || exit $?
EUNET_LIB=abl/liba3h3.so TAG=model_a3 TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_model.py tests/test_gpu_dual.py || exit $?
for L in abl/libgu1.so abl/libgu2.so; do
  EUNET_LIB=$L TAG=head_$(basename $L .so) TLIM=400 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "head" || exit $?
done
LIBS="abl/libb1h3.so abl/libp3h3.so abl/liba3h3.so" ROUNDS=2 bash tools/gpu_cb_libs.sh || exit $?
LIBS="abl/libgu1.so abl/libgu2.so abl/libgo2.so abl/libb1h3.so" REPS=10 TAG=gu bash tools/gpu_head_libs.sh || exit $?
for L in abl/libb1h3.so abl/liba3h3.so abl/libb1h3.so abl/liba3h3.so; do
  EUNET_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/r4h_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4h_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4h_bench.log | head -1) $(grep -o '"encoder_fwd": {"achieved": [0-9.]*, "frac": [0-9.]*' gpurun_out/r4h_bench.log)"
done
