#!/bin/bash
# round 4: conv epilogue (packed stats / bias, mask-free sums) -- correctness, per-layer A/B vs the
# round-3 conv (abl/libr3.so), bench; plus the re-run of this round's new tests
set -u
TAG=ops TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py -k "conv3x3 or head_bf16_batch_stats" || exit $?
TAG=model TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_model.py || exit $?
TAG=cfgs2 TLIM=600 bash tools/gpu_run_tests.sh tests/test_gpu_configs.py -k "bn_running" || exit $?
TAG=dp2b TLIM=700 bash tools/gpu_run_tests.sh tests/test_dp_gpu.py -k "trainer_steps or mean_of_shards" || exit $?
LIBS="abl/libr3.so enhanced-unet_amd/eunet/libeunet_hip.so" ROUNDS=2 bash tools/gpu_cb_libs.sh || exit $?
for L in abl/libr3.so ""; do
  EUNET_LIB_ALLOW_PARTIAL=1 EUNET_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/r4b_bench.log 2>&1 || exit $?
  echo "bench lib=${L:-new} $(grep -o '"value": [0-9.]*' gpurun_out/r4b_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4b_bench.log | head -1) $(grep -o '"encoder_fwd": {"achieved": [0-9.]*, "frac": [0-9.]*' gpurun_out/r4b_bench.log)"
done
