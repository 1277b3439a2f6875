#!/bin/bash
# round 4: conv epilogue step 2 (BNB template, row-strided store addresses, packed operand transform):
# correctness, A/B vs step 1 (abl/libe1.so), bench; re-runs of the fixed tests
set -u
TAG=ops TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "conv3x3" || exit $?
TAG=model TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_model.py tests/test_gpu_dual.py || exit $?
TAG=cfgs3 TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_configs.py -k "bn_running" || exit $?
TAG=dp2c TLIM=700 bash tools/gpu_run_tests.sh tests/test_dp_gpu.py -k "mean_of_shards" || exit $?
LIBS="abl/libe1.so enhanced-unet_amd/eunet/libeunet_hip.so" ROUNDS=2 bash tools/gpu_cb_libs.sh || exit $?
for L in abl/libe1.so "" abl/libe1.so ""; do
  EUNET_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/r4c_bench.log 2>&1 || exit $?
  echo "bench lib=${L:-new} $(grep -o '"value": [0-9.]*' gpurun_out/r4c_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4c_bench.log | head -1) $(grep -o '"encoder_fwd": {"achieved": [0-9.]*, "frac": [0-9.]*' gpurun_out/r4c_bench.log)"
done
