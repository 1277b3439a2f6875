#!/bin/bash
# round 4: conv halo layout / LDS-DMA variants vs B1+H3 (plane-major, register staging):
#  a5 = pixel-major (quarter XOR-swizzled) + halo DMA for untransformed forwards and plain dgrads
#  a7 = plane-major + halo DMA for plain dgrads only;  p5 = pixel-major swizzled, no halo DMA
#  wb5 / wb7 = a5 / a7 + the wgrad's in-place BN+ReLU reading 4 slots per LDS round trip
set -u
EUNET_LIB=abl/libwb5h3.so TAG=conv_wb5 TLIM=500 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "conv or dgrad" || exit $?
EUNET_LIB=abl/libwb7h3.so TAG=conv_wb7 TLIM=500 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "conv or dgrad" || exit $?
EUNET_LIB=abl/libwb5h3.so TAG=model_wb5 TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_model.py || exit $?
LIBS="abl/libb1h3.so abl/liba5h3.so abl/liba7h3.so abl/libp5h3.so abl/libwb5h3.so abl/libwb7h3.so" ROUNDS=2 bash tools/gpu_cb_libs.sh || exit $?
for L in abl/libb1h3.so abl/libwb5h3.so abl/libwb7h3.so abl/libb1h3.so abl/libwb5h3.so abl/libwb7h3.so; do
  EUNET_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/r4i_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4i_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4i_bench.log | head -1) $(grep -o '"encoder_fwd": {"achieved": [0-9.]*, "frac": [0-9.]*' gpurun_out/r4i_bench.log)"
done
