#!/bin/bash
# round 4: L1 = forward plane-major / register staging, plain data gradient pixel-major + halo LDS-DMA, wgrad
# transform reading 4 slots per LDS round trip (WB); L2 = L1 + the fused BN-backward reduction's constants in
# registers; vs B1+H3: parity, conv_bench, bench
set -u
EUNET_LIB=abl/libl2h3.so TAG=conv_l2 TLIM=500 bash tools/gpu_run_tests.sh tests/test_gpu_ops.py || exit $?
EUNET_LIB=abl/libl2h3.so TAG=model_l2 TLIM=700 bash tools/gpu_run_tests.sh tests/test_gpu_model.py tests/test_gpu_dual.py tests/test_gpu_configs.py || exit $?
LIBS="abl/libb1h3.so abl/libl1h3.so abl/libl2h3.so" ROUNDS=2 bash tools/gpu_cb_libs.sh || exit $?
for L in abl/libb1h3.so abl/libl2h3.so abl/libb1h3.so abl/libl2h3.so abl/libb1h3.so abl/libl2h3.so; do
  EUNET_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dice-size 0 --no-dp-world1 --no-fp32-leg > gpurun_out/r4j_bench.log 2>&1 || exit $?
  echo "bench lib=$L $(grep -o '"value": [0-9.]*' gpurun_out/r4j_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4j_bench.log | head -1) $(grep -o '"encoder_fwd": {"achieved": [0-9.]*, "frac": [0-9.]*' gpurun_out/r4j_bench.log)"
done
